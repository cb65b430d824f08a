function [xk, uk, Uk, exitflag, iters, wpred] = NTM_MPC_Sim_gpu(x0, k_sim, cfg, mode, gen)
%NTM_MPC_SIM_GPU  Drop-in for the controller loop of NTM_MPC_Sim.m (lines 80-131)
%   on MI355X, for one or many scenarios at once.
%
%   [xk, uk, Uk] = NTM_MPC_Sim_gpu(x0, k_sim, cfg)
%     x0    2-by-B initial states [w; omega], one column per scenario
%           (the reference's x0, NTM_MPC_Sim.m:34, is the B = 1 case)
%     k_sim number of time steps (NTM_MPC_Sim.m:80)
%     cfg   struct of controller settings (N, i_sim, mode, flags, Ts, xmin,
%           xmax, umin, umax, Q, r, epsilon, du_max, Ru); omitted fields take
%           the reference's literals (NTM_MPC_Sim.m:30-88).  du_max bounds the
%           input rate |U_i - U_{i-1}| in mode 3 (an extension, config 5); Ru
%           adds Ru*||U||^2 to the cost (the reference has none, Ru = 0);
%           flags selects the literal variants D4/D6/D13/D18 (SURVEY.md §2.1)
%     mode  'run' (default): the whole closed loop on the device, one call;
%           'step': one MEX call per time step (the state stays in MATLAB)
%     gen   optional scenario generator struct (seed, first_id, sigma_w,
%           sigma_omega, jbs_spread, wdep_spread): independent plasma
%           scenarios and plant disturbance realisations (ntm_scenario_gen);
%           omitted = the reference's nominal, disturbance-free loop
%   Returns the reference's workspace variables with a trailing scenario
%   dimension: xk 2-by-(k_sim+1)-by-B, uk 1-by-k_sim-by-B, Uk N-by-k_sim-by-B,
%   plus exitflag / iters (k_sim-by-B, quadprog codes and LPV iterations).
%
%   The MEX takes and returns E-by-B arrays (one column per scenario, the
%   ABI's scenario-major layout), so nothing is transposed on the way.
%
%   Semantics are the repaired ones of SURVEY.md §2.1 (CANON): Phi_i = A_i
%   Phi_{i-1}, Gamma_ij = A_i Gamma_{i-1,j}, W/L/c rebuilt each iteration, F
%   from the current x_k, plant step with +C, Uold = +Inf at start.
if nargin < 3, cfg = struct(); end
if nargin < 4, mode = 'run'; end
if nargin < 5, gen = []; end
if isempty(gen), ntm_mpc_mex('scenarios', []); else, ntm_mpc_mex('scenarios', gen); end
if ~isfield(cfg, 'N'), cfg.N = 20; end
N = cfg.N;
B = size(x0, 2);
switch mode
    case 'run'
        [XK, UK, UKK, WP, FL, IT] = ntm_mpc_mex('run', x0, k_sim, cfg);
        xk = reshape(XK, 2, k_sim + 1, B);
        uk = reshape(UK, 1, k_sim, B);
        Uk = reshape(UKK, N, k_sim, B);
        wpred = reshape(WP, N + 1, k_sim, B);   % predicted island width per step (:110-117)
        exitflag = FL;
        iters = IT;
    case 'step'
        xk = zeros(2, k_sim + 1, B); uk = zeros(1, k_sim, B); Uk = zeros(N, k_sim, B);
        wpred = zeros(N + 1, k_sim, B);
        exitflag = zeros(k_sim, B, 'int32'); iters = zeros(k_sim, B, 'int32');
        xk(:, 1, :) = reshape(x0, 2, 1, B);
        [Rho, Uold] = ntm_mpc_mex('init', x0, cfg);   % Rho = repmat(rho(x0),1,N), Uold = +Inf
        WS = -ones(2 * (N + 1), B, 'int32');         % warm-start workspace, carried step to step
        X = x0;
        k0_base = 0;                                 % the caller's first time index, as 'run' uses it
        if ~isempty(gen) && isfield(gen, 'k0'), k0_base = gen.k0; end
        for k = 1:k_sim
            if ~isempty(gen)                         % the plant step's time index
                gen.k0 = k0_base + k - 1; ntm_mpc_mex('scenarios', gen);
            end
            [U, XP, Xn, fl, it, Rho, Uold, WS] = ntm_mpc_mex('step', X, Rho, Uold, cfg, WS);
            wpred(:, k, :) = reshape(XP(1:2:end, :), N + 1, 1, B);
            Uk(:, k, :) = reshape(U, N, 1, B);
            uk(1, k, :) = reshape(U(1, :), 1, 1, B);
            exitflag(k, :) = fl; iters(k, :) = it;
            X = Xn;
            xk(:, k + 1, :) = reshape(Xn, 2, 1, B);
        end
    otherwise
        error('ntm:arg', 'mode must be ''run'' or ''step''');
end
end
