// ntm_device.h — device-side building blocks of the batched LPV-MPC hot path
// (gfx950 / CDNA4).  One scenario is owned by a GROUP of P lanes of a wave
// (P = 16, 32 or 64; 64/P scenarios per wave).  Lane l of a group owns index
// l of every length-N vector (decision variable u_l, prediction step l).
// All per-scenario matrices live in the group's slice of LDS; cross-lane
// traffic is LDS broadcast reads plus ds_bpermute shuffles inside the group.
// Every control decision is a group reduction, so control flow is
// group-uniform and the 64/P groups of a wave may diverge freely.
//
// Reference map (file:line of the MATLAB reference):
//   rho_eval          rho1.m:2, rho2.m:2, rho3.m:2-3
//   lift_phase        A.m:2, B.m:2, Rho_to_PhiGammaLambda.m:17-52 (CANON D4/D6)
//   cost_phase        NTM_MPC_Sim.m:67-73, 120-121 (CANON D8/D12)
//   StructRows        getWLc.m:9-59 rows, never materialised (implicit rows)
//   gi_solve          quadprog call NTM_MPC_Sim.m:97 (Goldfarb-Idnani)
//   rollout_phase     NTM_MPC_Sim.m:110-117, 123-127
//   plant_phase       NTM_MPC_Sim.m:130 (CANON D13)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ntm_mpc.h"

namespace ntm {

// ---------------------------------------------------------------------------
// launch-constant problem description (derived on the host, see ntm_capi.hip)
// ---------------------------------------------------------------------------
struct Coef {
    double a11c;    // (4/3)(kappa rs/(0.82 tau_r)) Ts           A.m:2
    double za3;     // zeta * a^3 (D19, divides rho2*Ts)         A.m:2
    double a22;     // 1 - Ts/tau_E                              A.m:2
    double bc;      // kappa Ts eta_CD / w_dep                   B.m:2
    double C1, C2;  // NTM_MPC_Sim.m:37
    double wmarg2;  // w_marg^2                                  rho1.m:2
    double wdep;    // w_dep                                     rho3.m:2
    double Ts;
    int rho1_sq;    // D18 switch
};

struct Prob {
    Coef k;
    int N, i_sim, mode, flags;
    double xmin[2], xmax[2], umin, umax, Q[4], r[2], eps;
};

constexpr double kInf = __builtin_huge_val();

#define NTM_WSYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

// ---------------------------------------------------------------------------
// group collectives (width-P segments of the 64-lane wave)
// ---------------------------------------------------------------------------
template <int P>
__device__ __forceinline__ double gsum(double v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, P);
    return v;
}
template <int P>
__device__ __forceinline__ double gmax(double v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, P));
    return v;
}
template <int P>
__device__ __forceinline__ int gmaxi(int v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, P));
    return v;
}
template <int P>
__device__ __forceinline__ double gbcast(double v, int src) { return __shfl(v, src, P); }

// argmin over (v, id) with ties broken towards the smaller id; carries two
// payload doubles.  Identical result in every lane of the group.
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id, double& a, double& b) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) {
        double ov = __shfl_xor(v, o, P);
        int oid = __shfl_xor(id, o, P);
        double oa = __shfl_xor(a, o, P);
        double ob = __shfl_xor(b, o, P);
        if (ov < v || (ov == v && oid < id)) { v = ov; id = oid; a = oa; b = ob; }
    }
}
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) {
        double ov = __shfl_xor(v, o, P);
        int oid = __shfl_xor(id, o, P);
        if (ov < v || (ov == v && oid < id)) { v = ov; id = oid; }
    }
}

// ---------------------------------------------------------------------------
// L0 / L1: scheduling parameters and LPV coefficients
// ---------------------------------------------------------------------------
// rho1.m:2, rho2.m:2, rho3.m:2-3 (same operation order as the oracle)
__device__ __forceinline__ void rho_eval(const Coef& k, double w, double om,
                                         double& r1, double& r2, double& r3) {
    r1 = 1.0 / ((k.rho1_sq ? w * w : w) + k.wmarg2);
    r2 = (w * w) / om;
    double ws = w / k.wdep;
    r3 = (0.25 + 0.24 * ws) / (1 + 1.5 * ws + 0.43 * (ws * ws) + 0.64 * (ws * ws * ws));
}
// A.m:2 entries a11, a21 (a12 = 0, a22 = k.a22); B.m:2 as the column [b; 0] (D5)
__device__ __forceinline__ double coef_a11(const Coef& k, double r1) { return k.a11c * r1 + 1; }
__device__ __forceinline__ double coef_a21(const Coef& k, double r2) { return (r2 * k.Ts) / k.za3; }
__device__ __forceinline__ double coef_b(const Coef& k, double r3) { return k.bc * r3; }

// ---------------------------------------------------------------------------
// per-scenario LDS workspace (all offsets in doubles; see ws_doubles())
// ---------------------------------------------------------------------------
struct WS {
    int N, LDG, LDJ;
    double* rho;   // 3N   (3xN col-major)
    double* a11;   // N
    double* a21;   // N
    double* bb;    // N
    double* Phi;   // 4N   Phi_i (2x2 col-major) per step
    double* Lam;   // 2N
    double* e;     // 2N   free response Phi x_k + Lambda
    double* Gt;    // 2N x N col-major (LDG = 2N): Gamma, then Gamma*D
    double* J;     // N x LDJ row-major: GI factor J = L^{-T} Q
    double* R;     // N x LDJ col-major: G, its Cholesky, then the GI R factor
    double* rn;    // 2N   norms of the scaled state rows
    double* F;     // N
    double* D;     // N    Jacobi scaling
    double* V;     // N    scaled decision variables
    double* d;     // N
    double* np;    // N    GI normal of the constraint being added
    double* hv;    // N    Householder vector
    double* uu;    // N+1  multipliers
    double* xp;    // 2(N+1) rollout
    double* U;     // N
    double* Uold;  // N
    int* act;      // N+1  active rows (ids)
    unsigned char* aflag;  // MMAX  active flag per row id
};

__host__ __device__ inline int ldj_of(int N) { return N | 1; }
__host__ __device__ inline int ws_doubles(int N) {
    int LDJ = ldj_of(N);
    return 3 * N + 3 * N + 4 * N + 2 * N + 2 * N + 2 * N * N + 2 * N * LDJ + 2 * N + 6 * N +
           (N + 1) + 2 * (N + 1) + 2 * N;
}
__host__ __device__ inline int ws_bytes(int N) {
    int b = ws_doubles(N) * 8 + (N + 1) * 4 + (6 * NTM_MAX_N + 4);
    return (b + 15) & ~15;
}

__device__ inline WS ws_carve(char* base, int N) {
    WS w;
    w.N = N;
    w.LDG = 2 * N;
    w.LDJ = ldj_of(N);
    double* p = reinterpret_cast<double*>(base);
    w.rho = p; p += 3 * N;
    w.a11 = p; p += N;
    w.a21 = p; p += N;
    w.bb = p; p += N;
    w.Phi = p; p += 4 * N;
    w.Lam = p; p += 2 * N;
    w.e = p; p += 2 * N;
    w.Gt = p; p += 2 * N * N;
    w.J = p; p += N * w.LDJ;
    w.R = p; p += N * w.LDJ;
    w.rn = p; p += 2 * N;
    w.F = p; p += N;
    w.D = p; p += N;
    w.V = p; p += N;
    w.d = p; p += N;
    w.np = p; p += N;
    w.hv = p; p += N;
    w.uu = p; p += N + 1;
    w.xp = p; p += 2 * (N + 1);
    w.U = p; p += N;
    w.Uold = p; p += N;
    w.act = reinterpret_cast<int*>(p);
    w.aflag = reinterpret_cast<unsigned char*>(w.act + N + 1);
    return w;
}

// ---------------------------------------------------------------------------
// L2: lifted prediction  (Rho_to_PhiGammaLambda.m:17-52, CANON D4/D6)
// ---------------------------------------------------------------------------
template <int P>
__device__ void lift_phase(const Prob& pb, const WS& w, int l) {
    const int N = w.N;
    const Coef& k = pb.k;
    if (l < N) {
        w.a11[l] = coef_a11(k, w.rho[3 * l]);
        w.a21[l] = coef_a21(k, w.rho[3 * l + 1]);
        w.bb[l] = coef_b(k, w.rho[3 * l + 2]);
    }
    NTM_WSYNC();
    // Gamma: lane j owns column j: Gamma_jj = B_j, Gamma_ij = A_i Gamma_{i-1,j} (D6)
    if (l < N) {
        double* col = w.Gt + l * w.LDG;
        for (int r = 0; r < 2 * l; ++r) col[r] = 0.0;
        double g0 = w.bb[l], g1 = 0.0;
        col[2 * l] = g0;
        col[2 * l + 1] = g1;
        for (int i = l + 1; i < N; ++i) {
            double n0 = w.a11[i] * g0;
            double n1 = w.a21[i] * g0 + k.a22 * g1;
            g0 = n0;
            g1 = n1;
            col[2 * i] = g0;
            col[2 * i + 1] = g1;
        }
    }
    // Phi (left-multiplied, D4) and Lambda: short sequential chains on lane 0
    if (l == 0) {
        double p00 = w.a11[0], p10 = w.a21[0], p01 = 0.0, p11 = k.a22;
        double l0 = k.C1, l1 = k.C2;
        w.Phi[0] = p00; w.Phi[1] = p10; w.Phi[2] = p01; w.Phi[3] = p11;
        w.Lam[0] = l0; w.Lam[1] = l1;
        for (int i = 1; i < N; ++i) {
            double a11 = w.a11[i], a21 = w.a21[i];
            double q00 = a11 * p00, q01 = a11 * p01;
            double q10 = a21 * p00 + k.a22 * p10, q11 = a21 * p01 + k.a22 * p11;
            p00 = q00; p01 = q01; p10 = q10; p11 = q11;
            double m0 = a11 * l0 + k.C1;
            double m1 = (a21 * l0 + k.a22 * l1) + k.C2;
            l0 = m0; l1 = m1;
            w.Phi[4 * i] = p00; w.Phi[4 * i + 1] = p10; w.Phi[4 * i + 2] = p01; w.Phi[4 * i + 3] = p11;
            w.Lam[2 * i] = l0; w.Lam[2 * i + 1] = l1;
        }
    }
    NTM_WSYNC();
}

// free response e = Phi x_k + Lambda (the x-dependent part of NTM_MPC_Sim.m:121
// and of c + W x_k at :97)
template <int P>
__device__ void free_response(const WS& w, double x0, double x1, int l) {
    for (int i = l; i < w.N; i += P) {
        const double* Ph = w.Phi + 4 * i;
        w.e[2 * i] = (Ph[0] * x0 + Ph[2] * x1) + w.Lam[2 * i];
        w.e[2 * i + 1] = (Ph[1] * x0 + Ph[3] * x1) + w.Lam[2 * i + 1];
    }
    NTM_WSYNC();
}

// ---------------------------------------------------------------------------
// condensed cost G = 2 Gamma' Om Gamma (lower triangle into w.R, col-major),
// F = 2 Gamma' Om (e - R)      NTM_MPC_Sim.m:120-121 (CANON D8, D12)
// ---------------------------------------------------------------------------
template <int P>
__device__ void cost_phase(const Prob& pb, const WS& w, int l) {
    const int N = w.N, LD = w.LDJ, LDG = w.LDG;
    const double q00 = pb.Q[0], q01 = pb.Q[1], q10 = pb.Q[2], q11 = pb.Q[3];
    if (l < N) {
        const double* cj = w.Gt + l * LDG;
        for (int kk = 0; kk <= l; ++kk) {
            const double* ck = w.Gt + kk * LDG;
            double s = 0.0;
            for (int i = l; i < N; ++i) {
                double g0 = ck[2 * i], g1 = ck[2 * i + 1];
                double o0 = q00 * g0 + q01 * g1;
                double o1 = q10 * g0 + q11 * g1;
                s += cj[2 * i] * o0;
                s += cj[2 * i + 1] * o1;
            }
            w.R[l + kk * LD] = 2 * s;   // G(l, kk), l >= kk
        }
        double f = 0.0;
        for (int i = l; i < N; ++i) {
            double e0 = w.e[2 * i] - pb.r[0], e1 = w.e[2 * i + 1] - pb.r[1];
            double o0 = q00 * e0 + q01 * e1;
            double o1 = q10 * e0 + q11 * e1;
            f += cj[2 * i] * o0 + cj[2 * i + 1] * o1;
        }
        w.F[l] = 2 * f;
    }
    NTM_WSYNC();
}

// ---------------------------------------------------------------------------
// Jacobi scaling U = D V: G~ = D G D, F~ = D F, Gamma~ = Gamma D, row norms.
// Returns false (group-uniform) if any datum is non-finite.
// ---------------------------------------------------------------------------
template <int P>
__device__ bool scale_phase(const WS& w, int l, bool with_state_rows) {
    const int N = w.N, LD = w.LDJ, LDG = w.LDG;
    if (l < N) {
        double g = w.R[l + l * LD];
        w.D[l] = (g > 0.0) ? 1.0 / sqrt(g) : 1.0;
    }
    NTM_WSYNC();
    int bad = 0;
    if (l < N) {
        double Dl = w.D[l];
        for (int kk = 0; kk <= l; ++kk) {
            double v = w.R[l + kk * LD] * Dl * w.D[kk];
            bad |= !isfinite(v);
            w.R[l + kk * LD] = v;
        }
        double f = w.F[l] * Dl;
        bad |= !isfinite(f);
        w.F[l] = f;
        if (with_state_rows) {
            double* col = w.Gt + l * LDG;
            for (int r = 2 * l; r < 2 * N; ++r) col[r] *= Dl;
        }
    }
    NTM_WSYNC();
    if (with_state_rows) {
        for (int r = l; r < 2 * N; r += P) {
            double s = 0.0;
            int jmax = r >> 1;
            for (int j = 0; j <= jmax; ++j) { double v = w.Gt[r + j * LDG]; s += v * v; }
            bad |= !isfinite(s) || !isfinite(w.e[r]);
            w.rn[r] = s > 0.0 ? sqrt(s) : 0.0;
        }
        NTM_WSYNC();
    }
    return gmaxi<P>(bad) == 0;
}

// ---------------------------------------------------------------------------
// Constraint-row providers for the dual active-set solver.  Row ids follow
// the oracle: box mode rows 0..N-1 are u_j >= umin, N..2N-1 are u_j <= umax;
// full mode rows follow getWLc.m:9-59 block by block (6 per step, 4 terminal).
// ---------------------------------------------------------------------------
struct Pick {
    int p;        // row id (-1 none)
    double s;     // normalised slack (GI form n'V - bc)
    double bc;    // normalised GI right-hand side
};

// Implicit getWLc rows: u-bounds are +-e_j, state rows are +-Gamma~_r / rn_r.
struct StructRows {
    const Prob* pb;
    int mode;     // NTM_MODE_BOX or NTM_MODE_FULL (NONE never constructs rows)

    __device__ int rows() const { return mode == NTM_MODE_BOX ? 2 * pb->N : 6 * pb->N + 4; }

    // constant rows (x_0 rows; state rows with Gamma_r == 0): 0 <= b or infeasible (D15)
    template <int P>
    __device__ bool feasible_const(const WS& w, double x0, double x1, int l) const {
        int bad = 0;
        if (mode == NTM_MODE_FULL) {
            if (l == 0) {
                bad |= (x0 - pb->xmin[0]) < 0.0;
                bad |= (x1 - pb->xmin[1]) < 0.0;
                bad |= (pb->xmax[0] - x0) < 0.0;
                bad |= (pb->xmax[1] - x1) < 0.0;
            }
            for (int r = l; r < 2 * w.N; r += P) {
                if (w.rn[r] == 0.0) {
                    int c = r & 1;
                    bad |= (w.e[r] - pb->xmin[c]) < 0.0;
                    bad |= (pb->xmax[c] - w.e[r]) < 0.0;
                }
            }
        }
        return gmaxi<P>(bad) == 0;
    }

    template <int P>
    __device__ Pick check(const WS& w, double Vl, int l) const {
        const int N = w.N;
        double bv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff;
        auto consider = [&](double s, int id, double bcv) {
            if (!w.aflag[id] && (s < bv || (s == bv && id < bid))) { bv = s; bid = id; bs = s; bbc = bcv; }
        };
        if (l < N) {
            double Dl = w.D[l];
            double lo = -((-pb->umin) / Dl);
            double hi = pb->umax / Dl;
            int idl = (mode == NTM_MODE_BOX) ? l : 6 * l;
            int idh = (mode == NTM_MODE_BOX) ? N + l : 6 * l + 1;
            consider(Vl - lo, idl, lo);
            consider(hi - Vl, idh, -hi);
        }
        if (mode == NTM_MODE_FULL) {
            for (int r = l; r < 2 * N; r += P) {
                double rnr = w.rn[r];
                if (rnr > 0.0) {
                    int jmax = r >> 1;
                    double xh = 0.0;
                    for (int j = 0; j <= jmax; ++j) xh += w.Gt[r + j * w.LDG] * w.V[j];
                    xh += w.e[r];
                    int c = r & 1, i = jmax + 1;
                    int idmin = (i < N) ? 6 * i + 2 + c : 6 * N + c;
                    double bmin = (w.e[r] - pb->xmin[c]) / rnr;     // |b| of the min row
                    double bmax = (pb->xmax[c] - w.e[r]) / rnr;
                    consider((xh - pb->xmin[c]) / rnr, idmin, -bmin);
                    consider((pb->xmax[c] - xh) / rnr, idmin + 2, -bmax);
                }
            }
        }
        gargmin<P>(bv, bid, bs, bbc);
        Pick pk;
        pk.p = (bv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }

    // GI normal n_p (= -Lin_p scaled+normalised) into w.np; returns bc_p
    template <int P>
    __device__ double load_np(const WS& w, int p, int l) const {
        const int N = w.N;
        double bc;
        if (mode == NTM_MODE_BOX) {
            int j = p < N ? p : p - N;
            bool upper = p >= N;
            if (l < N) w.np[l] = (l == j) ? (upper ? -1.0 : 1.0) : 0.0;
            double Dj = w.D[j];
            bc = upper ? -(pb->umax / Dj) : -((-pb->umin) / Dj);
        } else {
            int blk = p / 6, rr = p - 6 * blk;
            if (blk < N && rr < 2) {
                bool upper = rr == 1;
                if (l < N) w.np[l] = (l == blk) ? (upper ? -1.0 : 1.0) : 0.0;
                double Dj = w.D[blk];
                bc = upper ? -(pb->umax / Dj) : -((-pb->umin) / Dj);
            } else {
                int i, c;
                bool upper;
                if (blk < N) { i = blk; c = (rr - 2) & 1; upper = rr >= 4; }
                else { i = N; c = rr & 1; upper = rr >= 2; }
                int r = 2 * (i - 1) + c;
                double rnr = w.rn[r];
                double sg = upper ? -1.0 : 1.0;
                if (l < N) w.np[l] = (l <= (r >> 1)) ? sg * (w.Gt[r + l * w.LDG] / rnr) : 0.0;
                bc = upper ? -((pb->xmax[c] - w.e[r]) / rnr) : ((pb->xmin[c] - w.e[r]) / rnr);
            }
        }
        NTM_WSYNC();
        return bc;
    }
};

// Explicit dense rows Lin U <= b (batched SoA in global memory) for the
// quadprog-level entry point ntm_qp_device.
struct DenseRows {
    const double* Lin;  // element (i, j) of scenario s at [(i + j*m)*B + s]
    const double* b;    // [i*B + s]
    double* rnrm;       // LDS, m entries
    int64_t B, s;
    int m;

    __device__ int rows() const { return m; }
    __device__ double L(int i, int j) const { return Lin[((int64_t)i + (int64_t)j * m) * B + s]; }
    __device__ double bv(int i) const { return b[(int64_t)i * B + s]; }

    template <int P>
    __device__ bool prepare(const WS& w, int l) {
        int bad = 0;
        for (int i = l; i < m; i += P) {
            double ss = 0.0;
            for (int j = 0; j < w.N; ++j) { double v = L(i, j) * w.D[j]; ss += v * v; }
            double bi = bv(i);
            bad |= !isfinite(ss) || !isfinite(bi);
            rnrm[i] = ss > 0.0 ? sqrt(ss) : 0.0;
            if (!(ss > 0.0) && bi < 0.0) bad |= 2;
        }
        NTM_WSYNC();
        return gmaxi<P>(bad) == 0;
    }
    template <int P>
    __device__ int prepare_code(const WS& w, int l) {
        int bad = 0;
        for (int i = l; i < m; i += P) {
            double ss = 0.0;
            for (int j = 0; j < w.N; ++j) { double v = L(i, j) * w.D[j]; ss += v * v; }
            double bi = bv(i);
            if (!isfinite(ss) || !isfinite(bi)) bad |= 1;
            rnrm[i] = ss > 0.0 ? sqrt(ss) : 0.0;
            if (!(ss > 0.0) && bi < 0.0) bad |= 2;
        }
        NTM_WSYNC();
        return gmaxi<P>(bad);
    }
    template <int P>
    __device__ Pick check(const WS& w, double Vl, int l) const {
        double bvv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff;
        for (int i = l; i < m; i += P) {
            double rn = rnrm[i];
            if (rn > 0.0 && !w.aflag[i]) {
                double s = 0.0;
                for (int j = 0; j < w.N; ++j) s -= ((L(i, j) * w.D[j]) / rn) * w.V[j];
                double bi = bv(i) / rn;
                s += bi;
                if (s < bvv || (s == bvv && i < bid)) { bvv = s; bid = i; bs = s; bbc = -bi; }
            }
        }
        gargmin<P>(bvv, bid, bs, bbc);
        Pick pk;
        pk.p = (bvv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }
    template <int P>
    __device__ double load_np(const WS& w, int p, int l) const {
        double rn = rnrm[p];
        if (l < w.N) w.np[l] = -((L(p, l) * w.D[l]) / rn);
        NTM_WSYNC();
        return -(bv(p) / rn);
    }
};

// ---------------------------------------------------------------------------
// Goldfarb-Idnani dual active set on the Jacobi-scaled problem.
//   min 1/2 V'G~V + F~'V  s.t.  n_i'V >= bc_i (rows from the provider)
// Pre:  w.R holds G~ (lower, col-major), w.F holds F~, w.aflag cleared.
// Post: w.V holds V; returns the quadprog exit flag.  Adds use a Householder
// reflector on J's trailing columns (one reduction instead of a Givens chain);
// drops restore R with a Givens sweep (GI 1983, section 3).
// ---------------------------------------------------------------------------
template <int P, class Rows>
__device__ int gi_solve(const WS& w, const Rows* rows, int nrows, int l, int* iters_out) {
    const int N = w.N, LD = w.LDJ, LDJ = w.LDJ;
    *iters_out = 0;
    // 1. Cholesky G~ = L L' (left-looking, in place in w.R)
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        if (l >= k && l < N) {
            s = w.R[l + k * LD];
            for (int j = 0; j < k; ++j) s -= w.R[l + j * LD] * w.R[k + j * LD];
        }
        double dk = gbcast<P>(s, k);
        if (!(dk > 0.0)) return NTM_EXIT_NONFINITE;
        double lk = sqrt(dk);
        if (l > k && l < N) w.R[l + k * LD] = s / lk;
        if (l == k) w.R[k + k * LD] = lk;
        NTM_WSYNC();
    }
    // 2. J = L^{-T}: lane c computes row c of J (= column c of L^{-1})
    if (l < N) {
        for (int i = 0; i < N; ++i) {
            double x = 0.0;
            if (i >= l) {
                x = (i == l) ? 1.0 : 0.0;
                for (int k2 = l; k2 < i; ++k2) x -= w.R[i + k2 * LD] * w.J[l * LDJ + k2];
                x /= w.R[i + i * LD];
            }
            w.J[l * LDJ + i] = x;
        }
    }
    NTM_WSYNC();
    // 3. unconstrained minimiser V = -J J' F~
    double Vl = 0.0;
    {
        double t = 0.0;
        if (l < N) for (int i = 0; i < N; ++i) t += w.J[i * LDJ + l] * w.F[i];
        if (l < N) w.d[l] = t;
        NTM_WSYNC();
        if (l < N) {
            double v = 0.0;
            for (int k2 = 0; k2 < N; ++k2) v += w.J[l * LDJ + k2] * w.d[k2];
            Vl = -v;
            w.V[l] = Vl;
        }
        NTM_WSYNC();
    }
    if (!rows) return NTM_EXIT_OPTIMAL;
    const int max_iter = 10 * (N + nrows) + 50;
    int q = 0, it = 0;
    for (;;) {
        Pick pk = rows->template check<P>(w, Vl, l);
        if (pk.p < 0) { *iters_out = it; return NTM_EXIT_OPTIMAL; }
        double vmax = gmax<P>(l < N ? fabs(Vl) : 0.0);
        double tol = 1e-12 * fmax(fmax(1.0, vmax), fabs(pk.bc));
        if (pk.s >= -tol) { *iters_out = it; return NTM_EXIT_OPTIMAL; }
        const int p = pk.p;
        const double bcp = rows->template load_np<P>(w, p, l);
        double upq = 0.0;   // multiplier of the constraint being added
        for (;;) {
            if (++it > max_iter) { *iters_out = it; return NTM_EXIT_MAXITER; }
            // d = J' n_p
            double dl = 0.0;
            if (l < N) for (int i = 0; i < N; ++i) dl += w.J[i * LDJ + l] * w.np[i];
            if (l < N) w.d[l] = dl;
            NTM_WSYNC();
            // z = J2 d2 (primal direction)
            double zl = 0.0;
            if (l < N) for (int k2 = q; k2 < N; ++k2) zl += w.J[l * LDJ + k2] * w.d[k2];
            // r = R^{-1} d1 (negative dual direction), back substitution
            double acc = (l < q) ? dl : 0.0, rl = 0.0;
            for (int b = q - 1; b >= 0; --b) {
                double rb = gbcast<P>(acc, b) / w.R[b + b * LD];
                if (l == b) rl = rb;
                if (l < b) acc -= w.R[l + b * LD] * rb;
            }
            // partial (dual) step length t1
            double ratio = (l < q && rl > 0.0) ? w.uu[l] / rl : kInf;
            int li = l;
            gargmin<P>(ratio, li);
            const double t1 = ratio;
            // full (primal) step length t2
            double npl = (l < N) ? w.np[l] : 0.0;
            double zn = gsum<P>(zl * npl);
            double sp = gsum<P>(npl * Vl) - bcp;
            double znrm = gsum<P>(zl * zl);
            double dnrm = gsum<P>(dl * dl);
            double t2 = (fabs(zn) <= 1e-300 || sqrt(znrm) <= 1e-14 * sqrt(dnrm)) ? kInf : -sp / zn;
            double t = fmin(t1, t2);
            if (!(t < kInf)) { *iters_out = it; return NTM_EXIT_INFEASIBLE; }
            if (l < q) w.uu[l] -= t * rl;
            upq += t;
            if (t2 < kInf) {
                Vl += t * zl;
                if (l < N) w.V[l] = Vl;
                if (t == t2) {
                    // ---- add p: Householder on d[q:N] -> J(:, q:N) ----
                    double dq2 = (l >= q && l < N) ? dl * dl : 0.0;
                    double nrm = sqrt(gsum<P>(dq2));
                    double dqv = gbcast<P>(dl, q);
                    double h = dqv;
                    if (q < N - 1 && nrm > 0.0) {
                        h = (dqv >= 0.0) ? -nrm : nrm;
                        double vl = (l == q) ? dl - h : ((l > q && l < N) ? dl : 0.0);
                        if (l < N) w.hv[l] = vl;
                        double vtv = gsum<P>(vl * vl);
                        NTM_WSYNC();
                        if (l < N) {
                            double dot = 0.0;
                            for (int k2 = q; k2 < N; ++k2) dot += w.J[l * LDJ + k2] * w.hv[k2];
                            double f = 2.0 * dot / vtv;
                            for (int k2 = q; k2 < N; ++k2) w.J[l * LDJ + k2] -= f * w.hv[k2];
                        }
                    }
                    if (l < q) w.R[l + q * LD] = dl;
                    if (l == q) {
                        w.R[q + q * LD] = h;
                        w.act[q] = p;
                        w.aflag[p] = 1;
                        w.uu[q] = upq;
                    }
                    ++q;
                    NTM_WSYNC();
                    break;
                }
            }
            // ---- drop active position li (partial or dual-only step) ----
            const int l0 = li;
            const int dropped = w.act[l0];
            NTM_WSYNC();
            if (l < q) {
                for (int c = l0; c < q - 1; ++c) w.R[l + c * LD] = w.R[l + (c + 1) * LD];
                w.R[l + (q - 1) * LD] = 0.0;
            }
            {
                int an = 0;
                double un = 0.0;
                if (l >= l0 && l < q) { an = w.act[l + 1]; un = w.uu[l + 1]; }
                NTM_WSYNC();
                if (l >= l0 && l < q) { w.act[l] = an; w.uu[l] = un; }
                if (l == 0) w.aflag[dropped] = 0;
            }
            NTM_WSYNC();
            for (int j = l0; j < q - 1; ++j) {
                double a = w.R[j + j * LD], bq = w.R[(j + 1) + j * LD];
                double hh = hypot(a, bq);
                double cc = 1.0, ss = 0.0;
                if (hh != 0.0) { cc = a / hh; ss = bq / hh; }
                NTM_WSYNC();
                if (l >= j && l < q - 1) {
                    double r1 = w.R[j + l * LD], r2 = w.R[(j + 1) + l * LD];
                    w.R[j + l * LD] = cc * r1 + ss * r2;
                    w.R[(j + 1) + l * LD] = (l == j) ? 0.0 : (-ss * r1 + cc * r2);
                }
                if (l < N) {
                    double j1 = w.J[l * LDJ + j], j2 = w.J[l * LDJ + j + 1];
                    w.J[l * LDJ + j] = cc * j1 + ss * j2;
                    w.J[l * LDJ + j + 1] = -ss * j1 + cc * j2;
                }
                NTM_WSYNC();
            }
            --q;
        }
    }
}

// ---------------------------------------------------------------------------
// rollout + scheduling update + convergence (NTM_MPC_Sim.m:110-117, 123-127)
// Returns (group-uniform) whether sum|Uold - U| < eps; updates Uold.
// ---------------------------------------------------------------------------
template <int P>
__device__ bool rollout_phase(const Prob& pb, const WS& w, double x0, double x1, int l) {
    const int N = w.N;
    const Coef& k = pb.k;
    if (l == 0) {
        double y0 = x0, y1 = x1;
        w.xp[0] = y0;
        w.xp[1] = y1;
        for (int i = 0; i < N; ++i) {
            double n0 = (w.a11[i] * y0 + w.bb[i] * w.U[i]) + k.C1;
            double n1 = (w.a21[i] * y0 + k.a22 * y1) + k.C2;
            y0 = n0;
            y1 = n1;
            w.xp[2 * i + 2] = y0;
            w.xp[2 * i + 3] = y1;
        }
    }
    NTM_WSYNC();
    double dsum = 0.0;
    if (l < N) {
        double r1, r2, r3;
        rho_eval(k, w.xp[2 * l], w.xp[2 * l + 1], r1, r2, r3);
        w.rho[3 * l] = r1;
        w.rho[3 * l + 1] = r2;
        w.rho[3 * l + 2] = r3;
        double u = w.U[l];
        dsum = fabs(w.Uold[l] - u);
        w.Uold[l] = u;
    }
    NTM_WSYNC();
    double s = gsum<P>(dsum);
    return s < pb.eps;
}

// plant step NTM_MPC_Sim.m:130 (CANON D13: plant = prediction model, + C)
__device__ __forceinline__ void plant_step(const Prob& pb, double x0, double x1, double u,
                                           double& n0, double& n1) {
    const Coef& k = pb.k;
    double r1, r2, r3;
    rho_eval(k, x0, x1, r1, r2, r3);
    double a11 = coef_a11(k, r1), a21 = coef_a21(k, r2), b = coef_b(k, r3);
    n0 = a11 * x0 + b * u;
    n1 = a21 * x0 + k.a22 * x1;
    if (!(pb.flags & NTM_LITERAL_PLANT_NO_C)) { n0 += k.C1; n1 += k.C2; }
}

// ---------------------------------------------------------------------------
// one inner iteration's QP: build -> scale -> GI -> unscale into w.U
// ---------------------------------------------------------------------------
template <int P>
__device__ int qp_phase(const Prob& pb, const WS& w, double x0, double x1, int l, int* qp_iters) {
    const int N = w.N;
    lift_phase<P>(pb, w, l);
    free_response<P>(w, x0, x1, l);
    cost_phase<P>(pb, w, l);
    const bool full = pb.mode == NTM_MODE_FULL;
    int flag;
    if (!scale_phase<P>(w, l, full)) {
        flag = NTM_EXIT_NONFINITE;
        *qp_iters = 0;
    } else {
        StructRows rows{&pb, pb.mode};
        const int nrows = (pb.mode == NTM_MODE_NONE) ? 0 : rows.rows();
        if (pb.mode != NTM_MODE_NONE) {
            for (int i = l; i < nrows; i += P) w.aflag[i] = 0;
            NTM_WSYNC();
        }
        if (pb.mode != NTM_MODE_NONE && !rows.template feasible_const<P>(w, x0, x1, l)) {
            flag = NTM_EXIT_INFEASIBLE;
            *qp_iters = 0;
        } else {
            flag = gi_solve<P, StructRows>(w, pb.mode == NTM_MODE_NONE ? nullptr : &rows, nrows, l,
                                           qp_iters);
        }
    }
    if (l < N) {
        double u = 0.0;
        if (flag == NTM_EXIT_OPTIMAL || flag == NTM_EXIT_MAXITER) u = w.V[l] * w.D[l];
        w.U[l] = u;
    }
    NTM_WSYNC();
    return flag;
}

}  // namespace ntm
