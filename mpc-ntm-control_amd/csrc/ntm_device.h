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
    int32_t* stats;   // optional per-scenario counters (4 x B, SoA): QP solves,
                      // GI iterations, final active rows, general (state) active rows
};

constexpr double kInf = __builtin_huge_val();
constexpr double kDepTol = 1e-8;   // GI linear-dependence threshold (oracle GI_DEP_TOL)

#define NTM_WSYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

// ---------------------------------------------------------------------------
// group collectives (width-P segments of the 64-lane wave)
//
// Butterflies run on DPP / permlane VALU ops, not ds_bpermute: quad_perm
// (xor 1, xor 2), row_half_mirror (pairs the quads of an 8-lane group),
// row_mirror (pairs the 8-lane halves of a row), v_permlane16_swap (pairs
// the 16-lane rows of a 32-lane group) and v_permlane32_swap (pairs the wave
// halves).  Every pairing step combines the two operands symmetrically, so
// each lane of a group ends with the bit-identical result and every control
// decision taken on it stays group-uniform.  Callers must be in
// group-uniform control flow (all P lanes active).
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    int2 a = __builtin_bit_cast(int2, v);
    a.x = __builtin_amdgcn_update_dpp(0, a.x, CTRL, 0xF, 0xF, false);
    a.y = __builtin_amdgcn_update_dpp(0, a.y, CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, a);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }

// (lower-row value, upper-row value) of a 16-lane (S=16) or 32-lane (S=32) pairing, same in both partners
template <int S>
__device__ __forceinline__ void pair_d(double v, double& lo, double& hi) {
    int2 a = __builtin_bit_cast(int2, v);
    int2 x, y;
    if constexpr (S == 16) {
        auto r0 = __builtin_amdgcn_permlane16_swap(a.x, a.x, false, false);
        auto r1 = __builtin_amdgcn_permlane16_swap(a.y, a.y, false, false);
        x.x = r0[0]; x.y = r1[0]; y.x = r0[1]; y.y = r1[1];
    } else {
        auto r0 = __builtin_amdgcn_permlane32_swap(a.x, a.x, false, false);
        auto r1 = __builtin_amdgcn_permlane32_swap(a.y, a.y, false, false);
        x.x = r0[0]; x.y = r1[0]; y.x = r0[1]; y.y = r1[1];
    }
    lo = __builtin_bit_cast(double, x);
    hi = __builtin_bit_cast(double, y);
}
template <int S>
__device__ __forceinline__ void pair_i(int v, int& lo, int& hi) {
    if constexpr (S == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        lo = r[0]; hi = r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        lo = r[0]; hi = r[1];
    }
}

template <int P>
__device__ __forceinline__ double gsum(double v) {
    v = v + dpp_d<0xB1>(v);                       // quad_perm [1,0,3,2]
    v = v + dpp_d<0x4E>(v);                       // quad_perm [2,3,0,1]
    if constexpr (P >= 8) v = v + dpp_d<0x141>(v);   // row_half_mirror
    if constexpr (P >= 16) v = v + dpp_d<0x140>(v);  // row_mirror
    if constexpr (P >= 32) { double a, b; pair_d<16>(v, a, b); v = a + b; }
    if constexpr (P >= 64) { double a, b; pair_d<32>(v, a, b); v = a + b; }
    return v;
}
template <int P>
__device__ __forceinline__ double gmax(double v) {
    v = fmax(v, dpp_d<0xB1>(v));
    v = fmax(v, dpp_d<0x4E>(v));
    if constexpr (P >= 8) v = fmax(v, dpp_d<0x141>(v));
    if constexpr (P >= 16) v = fmax(v, dpp_d<0x140>(v));
    if constexpr (P >= 32) { double a, b; pair_d<16>(v, a, b); v = fmax(a, b); }
    if constexpr (P >= 64) { double a, b; pair_d<32>(v, a, b); v = fmax(a, b); }
    return v;
}
template <int P>
__device__ __forceinline__ int gmaxi(int v) {
    v = max(v, dpp_i<0xB1>(v));
    v = max(v, dpp_i<0x4E>(v));
    if constexpr (P >= 8) v = max(v, dpp_i<0x141>(v));
    if constexpr (P >= 16) v = max(v, dpp_i<0x140>(v));
    if constexpr (P >= 32) { int a, b; pair_i<16>(v, a, b); v = max(a, b); }
    if constexpr (P >= 64) { int a, b; pair_i<32>(v, a, b); v = max(a, b); }
    return v;
}
template <int P>
__device__ __forceinline__ double gbcast(double v, int src) { return __shfl(v, src, P); }

// argmin over (v, id) with ties broken towards the smaller id; carries two
// payload doubles.  Identical result in every lane of the group.
__device__ __forceinline__ void amin_sel(double& v, int& id, double& a, double& b, double ov, int oid, double oa,
                                         double ob) {
    if (ov < v || (ov == v && oid < id)) { v = ov; id = oid; a = oa; b = ob; }
}
template <int CTRL>
__device__ __forceinline__ void amin_dpp(double& v, int& id, double& a, double& b) {
    amin_sel(v, id, a, b, dpp_d<CTRL>(v), dpp_i<CTRL>(id), dpp_d<CTRL>(a), dpp_d<CTRL>(b));
}
template <int S>
__device__ __forceinline__ void amin_pair(double& v, int& id, double& a, double& b) {
    double v0, v1, a0, a1, b0, b1;
    int i0, i1;
    pair_d<S>(v, v0, v1);
    pair_i<S>(id, i0, i1);
    pair_d<S>(a, a0, a1);
    pair_d<S>(b, b0, b1);
    v = v0; id = i0; a = a0; b = b0;
    amin_sel(v, id, a, b, v1, i1, a1, b1);
}
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id, double& a, double& b) {
    amin_dpp<0xB1>(v, id, a, b);
    amin_dpp<0x4E>(v, id, a, b);
    if constexpr (P >= 8) amin_dpp<0x141>(v, id, a, b);
    if constexpr (P >= 16) amin_dpp<0x140>(v, id, a, b);
    if constexpr (P >= 32) amin_pair<16>(v, id, a, b);
    if constexpr (P >= 64) amin_pair<32>(v, id, a, b);
}
template <int P>
__device__ __forceinline__ void gargmin(double& v, int& id) {
    double a = 0.0, b = 0.0;
    gargmin<P>(v, id, a, b);
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
    double* base;
    // double offsets of each array (N is launch-uniform, so these fold to scalar math)
    __device__ __forceinline__ int oJ() const { return 14 * N + 2 * N * N; }
    __device__ __forceinline__ int oR() const { return oJ() + N * LDJ; }
    __device__ __forceinline__ int oM() const { return oR() + N * LDJ; }
    __device__ __forceinline__ int oV() const { return oM() + N * LDJ; }   // start of the vector block
    __device__ __forceinline__ double* rho() const { return base; }                 // 3N (3xN col-major)
    __device__ __forceinline__ double* a11() const { return base + 3 * N; }         // N
    __device__ __forceinline__ double* a21() const { return base + 4 * N; }         // N
    __device__ __forceinline__ double* bb() const { return base + 5 * N; }          // N
    __device__ __forceinline__ double* Phi() const { return base + 6 * N; }         // 4N Phi_i (2x2 col-major)
    __device__ __forceinline__ double* Lam() const { return base + 10 * N; }        // 2N
    __device__ __forceinline__ double* e() const { return base + 12 * N; }          // 2N free response
    __device__ __forceinline__ double* Gt() const { return base + 14 * N; }         // 2N x N col-major Gamma
    __device__ __forceinline__ double* J() const { return base + oJ(); }            // N x LDJ row-major
    __device__ __forceinline__ double* R() const { return base + oR(); }            // N x LDJ col-major
    __device__ __forceinline__ double* M() const { return base + oM(); }            // N x LDJ col-major
    __device__ __forceinline__ double* rn() const { return base + oV(); }           // 2N state-row norms
    __device__ __forceinline__ double* F() const { return base + oV() + 2 * N; }    // N  F~
    __device__ __forceinline__ double* D() const { return base + oV() + 3 * N; }    // N  Jacobi scaling
    __device__ __forceinline__ double* V() const { return base + oV() + 4 * N; }    // N  scaled variables
    __device__ __forceinline__ double* d() const { return base + oV() + 5 * N; }    // N
    __device__ __forceinline__ double* np() const { return base + oV() + 6 * N; }   // N  GI normal
    __device__ __forceinline__ double* hv() const { return base + oV() + 7 * N; }   // N  Householder / polish
    __device__ __forceinline__ double* Vb() const { return base + oV() + 8 * N; }   // N  polish fixed (V)
    __device__ __forceinline__ double* Uf() const { return base + oV() + 9 * N; }   // N  polish fixed (U)
    __device__ __forceinline__ double* uu() const { return base + oV() + 10 * N; }  // N+1 multipliers
    __device__ __forceinline__ double* xp() const { return base + oV() + 11 * N + 1; }   // 2(N+1) rollout
    __device__ __forceinline__ double* U() const { return base + oV() + 13 * N + 3; }    // N
    __device__ __forceinline__ double* Uold() const { return base + oV() + 14 * N + 3; } // N
    __device__ __forceinline__ int* act() const { return reinterpret_cast<int*>(base + oV() + 15 * N + 3); }
    __device__ __forceinline__ int* sidx() const { return act() + N + 1; }
    __device__ __forceinline__ int* cand() const { return act() + 2 * (N + 1); }   // 2(N+1): last two active sets
    __device__ __forceinline__ unsigned char* fx() const {
        return reinterpret_cast<unsigned char*>(act() + 4 * (N + 1));
    }
    __device__ __forceinline__ unsigned char* aflag() const { return fx() + N; }
};

__host__ __device__ inline int ldj_of(int N) { return N | 1; }
__host__ __device__ inline int ws_doubles(int N) { return 14 * N + 2 * N * N + 3 * N * ldj_of(N) + 15 * N + 3; }
__host__ __device__ inline int ws_bytes(int N) {
    int b = ws_doubles(N) * 8 + 4 * (N + 1) * 4 + N + (6 * NTM_MAX_N + 4);
    return (b + 15) & ~15;
}

__device__ inline WS ws_carve(char* base, int N) {
    WS w;
    w.N = N;
    w.LDG = 2 * N;
    w.LDJ = ldj_of(N);
    w.base = reinterpret_cast<double*>(base);
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
        w.a11()[l] = coef_a11(k, w.rho()[3 * l]);
        w.a21()[l] = coef_a21(k, w.rho()[3 * l + 1]);
        w.bb()[l] = coef_b(k, w.rho()[3 * l + 2]);
    }
    NTM_WSYNC();
    // Gamma: lane j owns column j: Gamma_jj = B_j, Gamma_ij = A_i Gamma_{i-1,j} (D6)
    if (l < N) {
        double* col = w.Gt() + l * w.LDG;
        for (int r = 0; r < 2 * l; ++r) col[r] = 0.0;
        double g0 = w.bb()[l], g1 = 0.0;
        col[2 * l] = g0;
        col[2 * l + 1] = g1;
        for (int i = l + 1; i < N; ++i) {
            double n0 = w.a11()[i] * g0;
            double n1 = w.a21()[i] * g0 + k.a22 * g1;
            g0 = n0;
            g1 = n1;
            col[2 * i] = g0;
            col[2 * i + 1] = g1;
        }
    }
    // Phi (left-multiplied, D4) and Lambda: short sequential chains on lane 0
    if (l == 0) {
        double p00 = w.a11()[0], p10 = w.a21()[0], p01 = 0.0, p11 = k.a22;
        double l0 = k.C1, l1 = k.C2;
        w.Phi()[0] = p00; w.Phi()[1] = p10; w.Phi()[2] = p01; w.Phi()[3] = p11;
        w.Lam()[0] = l0; w.Lam()[1] = l1;
        for (int i = 1; i < N; ++i) {
            double a11 = w.a11()[i], a21 = w.a21()[i];
            double q00 = a11 * p00, q01 = a11 * p01;
            double q10 = a21 * p00 + k.a22 * p10, q11 = a21 * p01 + k.a22 * p11;
            p00 = q00; p01 = q01; p10 = q10; p11 = q11;
            double m0 = a11 * l0 + k.C1;
            double m1 = (a21 * l0 + k.a22 * l1) + k.C2;
            l0 = m0; l1 = m1;
            w.Phi()[4 * i] = p00; w.Phi()[4 * i + 1] = p10; w.Phi()[4 * i + 2] = p01; w.Phi()[4 * i + 3] = p11;
            w.Lam()[2 * i] = l0; w.Lam()[2 * i + 1] = l1;
        }
    }
    NTM_WSYNC();
}

// free response e = Phi x_k + Lambda (the x-dependent part of NTM_MPC_Sim.m:121
// and of c + W x_k at :97)
template <int P>
__device__ void free_response(const WS& w, double x0, double x1, int l) {
    for (int i = l; i < w.N; i += P) {
        const double* Ph = w.Phi() + 4 * i;
        w.e()[2 * i] = (Ph[0] * x0 + Ph[2] * x1) + w.Lam()[2 * i];
        w.e()[2 * i + 1] = (Ph[1] * x0 + Ph[3] * x1) + w.Lam()[2 * i + 1];
    }
    NTM_WSYNC();
}

// ---------------------------------------------------------------------------
// condensed cost G = 2 Gamma' Om Gamma (lower triangle into dst, col-major),
// F = 2 Gamma' Om (e - R)      NTM_MPC_Sim.m:120-121 (CANON D8, D12)
// ---------------------------------------------------------------------------
template <int P>
__device__ void gram_rows(const Prob& pb, const WS& w, double* dst, int l) {
    const int N = w.N, LD = w.LDJ, LDG = w.LDG;
    const double q00 = pb.Q[0], q01 = pb.Q[1], q10 = pb.Q[2], q11 = pb.Q[3];
    if (l < N) {
        const double* cj = w.Gt() + l * LDG;
        for (int kk = 0; kk <= l; ++kk) {
            const double* ck = w.Gt() + kk * LDG;
            double s = 0.0;
            for (int i = l; i < N; ++i) {
                double g0 = ck[2 * i], g1 = ck[2 * i + 1];
                double o0 = q00 * g0 + q01 * g1;
                double o1 = q10 * g0 + q11 * g1;
                s += cj[2 * i] * o0;
                s += cj[2 * i + 1] * o1;
            }
            dst[l + kk * LD] = 2 * s;   // G(l, kk), l >= kk
        }
    }
}

template <int P>
__device__ void cost_phase(const Prob& pb, const WS& w, int l) {
    const int N = w.N, LDG = w.LDG;
    const double q00 = pb.Q[0], q01 = pb.Q[1], q10 = pb.Q[2], q11 = pb.Q[3];
    gram_rows<P>(pb, w, w.R(), l);
    if (l < N) {
        const double* cj = w.Gt() + l * LDG;
        double f = 0.0;
        for (int i = l; i < N; ++i) {
            double e0 = w.e()[2 * i] - pb.r[0], e1 = w.e()[2 * i + 1] - pb.r[1];
            double o0 = q00 * e0 + q01 * e1;
            double o1 = q10 * e0 + q11 * e1;
            f += cj[2 * i] * o0 + cj[2 * i + 1] * o1;
        }
        w.F()[l] = 2 * f;
    }
    NTM_WSYNC();
}

// G~ = D G D in place (lower triangle, col-major); the same expression order
// is used when the polish recomputes G~ (so both copies are bit-identical).
template <int P>
__device__ int scale_gram(const WS& w, double* G, int l) {
    int bad = 0;
    if (l < w.N) {
        double Dl = w.D()[l];
        for (int kk = 0; kk <= l; ++kk) {
            double v = G[l + kk * w.LDJ] * Dl * w.D()[kk];
            bad |= !isfinite(v);
            G[l + kk * w.LDJ] = v;
        }
    }
    return bad;
}

// ---------------------------------------------------------------------------
// Jacobi scaling U = D V: G~ = D G D, F~ = D F, norms of the scaled state rows
// ||Gamma_r D||.  Gamma itself stays unscaled (D is applied on the fly).
// Returns false (group-uniform) if any datum is non-finite.
// ---------------------------------------------------------------------------
template <int P>
__device__ bool scale_phase(const WS& w, int l, bool with_state_rows) {
    const int N = w.N, LD = w.LDJ, LDG = w.LDG;
    if (l < N) {
        double g = w.R()[l + l * LD];
        w.D()[l] = (g > 0.0) ? 1.0 / sqrt(g) : 1.0;
    }
    NTM_WSYNC();
    int bad = scale_gram<P>(w, w.R(), l);
    if (l < N) {
        double f = w.F()[l] * w.D()[l];
        bad |= !isfinite(f);
        w.F()[l] = f;
    }
    if (with_state_rows) {
        for (int r = l; r < 2 * N; r += P) {
            double s = 0.0;
            int jmax = r >> 1;
            for (int j = 0; j <= jmax; ++j) { double v = w.Gt()[r + j * LDG] * w.D()[j]; s += v * v; }
            bad |= !isfinite(s) || !isfinite(w.e()[r]);
            w.rn()[r] = s > 0.0 ? sqrt(s) : 0.0;
        }
    }
    NTM_WSYNC();
    return gmaxi<P>(bad) == 0;
}

// ---------------------------------------------------------------------------
// Constraint-row providers (Lin U <= b form, getWLc.m row convention).  Row
// ids follow the oracle: box mode rows 0..N-1 are u_j >= umin, N..2N-1 are
// u_j <= umax; full mode rows follow getWLc.m:9-59 block by block (6 per
// step, 4 terminal).  In the solver each row is scaled and normalised:
//   GI normal n = -(Lin D)/rn,  GI rhs bc = -b/rn,  slack s = n'V - bc.
// ---------------------------------------------------------------------------
struct Pick {
    int p;        // row id (-1 none)
    double s;     // normalised slack (GI form n'V - bc)
    double bc;    // normalised GI right-hand side
};

// Implicit getWLc rows: u-bounds are -+e_j, state rows are -+Gamma_r; the
// rows are never materialised.
struct StructRows {
    int N, mode;  // mode: NTM_MODE_BOX or NTM_MODE_FULL (NONE: no rows)
    double umin, umax, xmin0, xmin1, xmax0, xmax1;

    __device__ StructRows(const Prob& p)
        : N(p.N), mode(p.mode), umin(p.umin), umax(p.umax), xmin0(p.xmin[0]), xmin1(p.xmin[1]),
          xmax0(p.xmax[0]), xmax1(p.xmax[1]) {}
    __device__ __forceinline__ double xmin(int c) const { return c ? xmin1 : xmin0; }
    __device__ __forceinline__ double xmax(int c) const { return c ? xmax1 : xmax0; }

    __device__ int rows() const { return mode == NTM_MODE_BOX ? 2 * N : 6 * N + 4; }

    // decode a row id: kind 0 = u lower, 1 = u upper, 2 = state min, 3 = state max;
    // j = variable (u rows) or state row r (state rows); -1 for x_0 rows
    __device__ void decode(int id, int N, int& kind, int& j) const {
        if (mode == NTM_MODE_BOX) {
            kind = id < N ? 0 : 1;
            j = id < N ? id : id - N;
            return;
        }
        int blk = id / 6, rr = id - 6 * blk;
        if (blk < N && rr < 2) { kind = rr; j = blk; return; }
        int i, c;
        bool upper;
        if (blk < N) { i = blk; c = (rr - 2) & 1; upper = rr >= 4; }
        else { i = N; c = rr & 1; upper = rr >= 2; }
        kind = upper ? 3 : 2;
        j = (i == 0) ? -1 : 2 * (i - 1) + c;
    }
    __device__ double lin(const WS& w, int id, int col) const {          // Lin[id][col]
        int kind, j;
        decode(id, w.N, kind, j);
        if (kind < 2) return (col == j) ? (kind == 0 ? -1.0 : 1.0) : 0.0;
        if (j < 0 || col > (j >> 1)) return 0.0;
        double g = w.Gt()[j + col * w.LDG];
        return kind == 2 ? -g : g;
    }
    __device__ double bval(const WS& w, int id) const {                  // b[id]
        int kind, j;
        decode(id, w.N, kind, j);
        if (kind == 0) return -umin;
        if (kind == 1) return umax;
        int c = j & 1;
        return kind == 2 ? (-xmin(c) + w.e()[j]) : (xmax(c) - w.e()[j]);
    }
    __device__ double rnorm(const WS& w, int id) const {
        int kind, j;
        decode(id, w.N, kind, j);
        return kind < 2 ? w.D()[j] : w.rn()[j];
    }

    // constant rows (x_0 rows; state rows with Gamma_r == 0): 0 <= b or infeasible (D15)
    template <int P>
    __device__ bool feasible_const(const WS& w, double x0, double x1, int l) const {
        int bad = 0;
        if (mode == NTM_MODE_FULL) {
            if (l == 0) {
                bad |= (x0 - xmin(0)) < 0.0;
                bad |= (x1 - xmin(1)) < 0.0;
                bad |= (xmax(0) - x0) < 0.0;
                bad |= (xmax(1) - x1) < 0.0;
            }
            for (int r = l; r < 2 * w.N; r += P) {
                if (w.rn()[r] == 0.0) {
                    int c = r & 1;
                    bad |= (w.e()[r] - xmin(c)) < 0.0;
                    bad |= (xmax(c) - w.e()[r]) < 0.0;
                }
            }
        }
        return gmaxi<P>(bad) == 0;
    }

    // Most violated inactive row (verify = false), or, with verify = true,
    // whether EVERY row has slack >= -tol * max(vmax, |bc|) (returned in .p).
    template <int P>
    __device__ Pick check(const WS& w, double Vl, int l, bool verify = false, double vmax = 1.0) const {
        const int N = w.N;
        if (mode == NTM_MODE_NONE) { Pick none; none.p = verify ? 0 : -1; none.s = 0.0; none.bc = 0.0; return none; }
        double bv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff, bad = 0;
        auto consider = [&](double s, int id, double bcv) {
            if (verify) { bad |= s < -1e-9 * fmax(vmax, fabs(bcv)); return; }
            if (!w.aflag()[id] && (s < bv || (s == bv && id < bid))) { bv = s; bid = id; bs = s; bbc = bcv; }
        };
        if (l < N) {
            double Dl = w.D()[l];
            double lo = -((-umin) / Dl);
            double hi = umax / Dl;
            int idl = (mode == NTM_MODE_BOX) ? l : 6 * l;
            int idh = (mode == NTM_MODE_BOX) ? N + l : 6 * l + 1;
            consider(Vl - lo, idl, lo);
            consider(hi - Vl, idh, -hi);
        }
        if (mode == NTM_MODE_FULL) {
            for (int r = l; r < 2 * N; r += P) {
                double rnr = w.rn()[r];
                if (rnr > 0.0) {
                    int jmax = r >> 1;
                    double xh = 0.0;
                    for (int j = 0; j <= jmax; ++j) xh += w.Gt()[r + j * w.LDG] * (w.D()[j] * w.V()[j]);
                    xh += w.e()[r];
                    int c = r & 1, i = jmax + 1;
                    int idmin = (i < N) ? 6 * i + 2 + c : 6 * N + c;
                    double bcmin = (xmin(c) - w.e()[r]) / rnr;
                    double bcmax = -((xmax(c) - w.e()[r]) / rnr);
                    consider((xh - xmin(c)) / rnr, idmin, bcmin);
                    consider((xmax(c) - xh) / rnr, idmin + 2, bcmax);
                }
            }
        }
        Pick pk;
        if (verify) {
            pk.p = gmaxi<P>(bad);
            pk.s = 0.0;
            pk.bc = 0.0;
            return pk;
        }
        gargmin<P>(bv, bid, bs, bbc);
        pk.p = (bv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }

    // GI normal n_p into w.np(); returns bc_p
    template <int P>
    __device__ double load_np(const WS& w, int p, int l) const {
        double rn = rnorm(w, p);
        if (l < w.N) w.np()[l] = -((lin(w, p, l) * w.D()[l]) / rn);
        NTM_WSYNC();
        return -(bval(w, p) / rn);
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
    __device__ double lin(const WS&, int i, int j) const { return Lin[((int64_t)i + (int64_t)j * m) * B + s]; }
    __device__ double bval(const WS&, int i) const { return b[(int64_t)i * B + s]; }
    __device__ double rnorm(const WS&, int i) const { return rnrm[i]; }

    template <int P>
    __device__ int prepare_code(const WS& w, int l) {
        int bad = 0;
        for (int i = l; i < m; i += P) {
            double ss = 0.0;
            for (int j = 0; j < w.N; ++j) { double v = lin(w, i, j) * w.D()[j]; ss += v * v; }
            double bi = bval(w, i);
            if (!isfinite(ss) || !isfinite(bi)) bad |= 1;
            rnrm[i] = ss > 0.0 ? sqrt(ss) : 0.0;
            if (!(ss > 0.0) && bi < 0.0) bad |= 2;
        }
        NTM_WSYNC();
        return gmaxi<P>(bad);
    }
    template <int P>
    __device__ Pick check(const WS& w, double Vl, int l, bool verify = false, double vmax = 1.0) const {
        double bvv = kInf, bs = 0.0, bbc = 0.0;
        int bid = 0x7fffffff, bad = 0;
        for (int i = l; i < m; i += P) {
            double rn = rnrm[i];
            if (rn > 0.0 && (verify || !w.aflag()[i])) {
                double sl = 0.0;
                for (int j = 0; j < w.N; ++j) sl -= ((lin(w, i, j) * w.D()[j]) / rn) * w.V()[j];
                double bi = bval(w, i) / rn;
                sl += bi;
                if (verify) bad |= sl < -1e-9 * fmax(vmax, fabs(bi));
                else if (sl < bvv || (sl == bvv && i < bid)) { bvv = sl; bid = i; bs = sl; bbc = -bi; }
            }
        }
        Pick pk;
        if (verify) {
            pk.p = gmaxi<P>(bad);
            pk.s = 0.0;
            pk.bc = 0.0;
            return pk;
        }
        gargmin<P>(bvv, bid, bs, bbc);
        pk.p = (bvv < kInf) ? bid : -1;
        pk.s = bs;
        pk.bc = bbc;
        return pk;
    }
    template <int P>
    __device__ double load_np(const WS& w, int p, int l) const {
        double rn = rnrm[p];
        if (l < w.N) w.np()[l] = -((lin(w, p, l) * w.D()[l]) / rn);
        NTM_WSYNC();
        return -(bval(w, p) / rn);
    }
};

// ---------------------------------------------------------------------------
// small dense kernels on a group's LDS matrices (col-major, leading dim LD)
// ---------------------------------------------------------------------------
// left-looking Cholesky of the n x n lower triangle of A, in place; false if not PD
template <int P>
__device__ bool chol_inplace(double* A, int n, int LD, int l) {
    for (int k = 0; k < n; ++k) {
        double s = 0.0;
        if (l >= k && l < n) {
            s = A[l + k * LD];
            for (int j = 0; j < k; ++j) s -= A[l + j * LD] * A[k + j * LD];
        }
        double dk = gbcast<P>(s, k);
        if (!(dk > 0.0)) return false;
        double lk = sqrt(dk);
        if (l > k && l < n) A[l + k * LD] = s / lk;
        if (l == k) A[k + k * LD] = lk;
        NTM_WSYNC();
    }
    return true;
}
// lane i holds b_i in `v`; returns x_i of L x = b (L lower, col-major)
template <int P>
__device__ double fwd_lanes(const double* L, int n, int LD, double v, int l) {
    double acc = (l < n) ? v : 0.0, x = 0.0;
    for (int k = 0; k < n; ++k) {
        double xk = gbcast<P>(acc, k) / L[k + k * LD];
        if (l == k) x = xk;
        if (l > k && l < n) acc -= L[l + k * LD] * xk;
    }
    return x;
}
// lane i holds b_i in `v`; returns x_i of L' x = b (L lower, col-major)
template <int P>
__device__ double bwd_lanes(const double* L, int n, int LD, double v, int l) {
    double acc = (l < n) ? v : 0.0, x = 0.0;
    for (int k = n - 1; k >= 0; --k) {
        double xk = gbcast<P>(acc, k) / L[k + k * LD];
        if (l == k) x = xk;
        if (l < k) acc -= L[k + l * LD] * xk;
    }
    return x;
}

// ---------------------------------------------------------------------------
// Goldfarb-Idnani dual active set on the Jacobi-scaled problem.
//   min 1/2 V'G~V + F~'V  s.t.  n_i'V >= bc_i (rows from the provider)
// Pre:  w.R() holds G~ (lower, col-major), w.F() holds F~, w.aflag() cleared.
// Post: w.V() holds V, w.act()[0..*q_out) the active rows; returns the quadprog
// exit flag.  Adds use a Householder reflector on J's trailing columns (one
// reduction instead of a Givens chain); drops restore R with a Givens sweep
// (Goldfarb & Idnani 1983, section 3).
// ---------------------------------------------------------------------------
template <int P, class Rows>
__device__ int gi_solve(const WS& w, const Rows* rows, int nrows, int l, int* iters_out, int* q_out) {
    const int N = w.N, LD = w.LDJ, LDJ = w.LDJ;
    *iters_out = 0;
    *q_out = 0;
    // 1. Cholesky G~ = L L' (in place in w.R())
    if (!chol_inplace<P>(w.R(), N, LD, l)) return NTM_EXIT_NONFINITE;
    // 2. J = L^{-T}: lane c computes row c of J (= column c of L^{-1})
    if (l < N) {
        for (int i = 0; i < N; ++i) {
            double x = 0.0;
            if (i >= l) {
                x = (i == l) ? 1.0 : 0.0;
                for (int k2 = l; k2 < i; ++k2) x -= w.R()[i + k2 * LD] * w.J()[l * LDJ + k2];
                x /= w.R()[i + i * LD];
            }
            w.J()[l * LDJ + i] = x;
        }
    }
    NTM_WSYNC();
    // 3. unconstrained minimiser V = -J J' F~
    double Vl = 0.0;
    {
        double t = 0.0;
        if (l < N) for (int i = 0; i < N; ++i) t += w.J()[i * LDJ + l] * w.F()[i];
        if (l < N) w.d()[l] = t;
        NTM_WSYNC();
        if (l < N) {
            double v = 0.0;
            for (int k2 = 0; k2 < N; ++k2) v += w.J()[l * LDJ + k2] * w.d()[k2];
            Vl = -v;
            w.V()[l] = Vl;
        }
        NTM_WSYNC();
    }
    if (!rows) return NTM_EXIT_OPTIMAL;
    const int max_iter = 10 * (N + nrows) + 50;
    int q = 0, it = 0;
    for (;;) {
        Pick pk = rows->template check<P>(w, Vl, l);
        double vmax = gmax<P>(l < N ? fabs(Vl) : 0.0);
        if (pk.p < 0 || pk.s >= -1e-12 * fmax(fmax(1.0, vmax), fabs(pk.bc))) {
            *iters_out = it;
            *q_out = q;
            return NTM_EXIT_OPTIMAL;
        }
        const int p = pk.p;
        const double bcp = rows->template load_np<P>(w, p, l);
        double upq = 0.0;   // multiplier of the constraint being added
        for (;;) {
            if (++it > max_iter) { *iters_out = it; *q_out = q; return NTM_EXIT_MAXITER; }
            // d = J' n_p
            double dl = 0.0;
            if (l < N) for (int i = 0; i < N; ++i) dl += w.J()[i * LDJ + l] * w.np()[i];
            if (l < N) w.d()[l] = dl;
            NTM_WSYNC();
            // z = J2 d2 (primal direction)
            double zl = 0.0;
            if (l < N) for (int k2 = q; k2 < N; ++k2) zl += w.J()[l * LDJ + k2] * w.d()[k2];
            // r = R^{-1} d1 (negative dual direction), back substitution
            double acc = (l < q) ? dl : 0.0, rl = 0.0;
            for (int b = q - 1; b >= 0; --b) {
                double rb = gbcast<P>(acc, b) / w.R()[b + b * LD];
                if (l == b) rl = rb;
                if (l < b) acc -= w.R()[l + b * LD] * rb;
            }
            // partial (dual) step length t1
            double ratio = (l < q && rl > 0.0) ? w.uu()[l] / rl : kInf;
            int li = l;
            gargmin<P>(ratio, li);
            const double t1 = ratio;
            // full (primal) step length t2.  z'n_p = |d2|^2 exactly (z = J2 d2),
            // never negative; n_p counts as dependent on the active rows when
            // |d2| <= kDepTol |d|
            double npl = (l < N) ? w.np()[l] : 0.0;
            double zn = gsum<P>((l >= q && l < N) ? dl * dl : 0.0);
            double sp = gsum<P>(npl * Vl) - bcp;
            double dnrm = gsum<P>(dl * dl);
            double t2 = (zn <= 1e-300 || sqrt(zn) <= kDepTol * sqrt(dnrm)) ? kInf : -sp / zn;
            double t = fmin(t1, t2);
            if (!(t < kInf)) { *iters_out = it; *q_out = q; return NTM_EXIT_INFEASIBLE; }
            if (l < q) w.uu()[l] = fmax(0.0, w.uu()[l] - t * rl);
            upq += t;
            if (t2 < kInf) {
                Vl += t * zl;
                if (l < N) w.V()[l] = Vl;
                if (t == t2) {
                    // ---- add p: Householder on d[q:N] -> J(:, q:N) ----
                    double dq2 = (l >= q && l < N) ? dl * dl : 0.0;
                    double nrm = sqrt(gsum<P>(dq2));
                    double dqv = gbcast<P>(dl, q);
                    double h = dqv;
                    if (q < N - 1 && nrm > 0.0) {
                        h = (dqv >= 0.0) ? -nrm : nrm;
                        double vl = (l == q) ? dl - h : ((l > q && l < N) ? dl : 0.0);
                        if (l < N) w.hv()[l] = vl;
                        double vtv = gsum<P>(vl * vl);
                        NTM_WSYNC();
                        if (l < N) {
                            double dot = 0.0;
                            for (int k2 = q; k2 < N; ++k2) dot += w.J()[l * LDJ + k2] * w.hv()[k2];
                            double f = 2.0 * dot / vtv;
                            for (int k2 = q; k2 < N; ++k2) w.J()[l * LDJ + k2] -= f * w.hv()[k2];
                        }
                    }
                    if (l < q) w.R()[l + q * LD] = dl;
                    if (l == q) {
                        w.R()[q + q * LD] = h;
                        w.act()[q] = p;
                        w.aflag()[p] = 1;
                        w.uu()[q] = upq;
                    }
                    ++q;
                    NTM_WSYNC();
                    break;
                }
            }
            // ---- drop active position li (partial or dual-only step) ----
            const int l0 = li;
            const int dropped = w.act()[l0];
            NTM_WSYNC();
            if (l < q) {
                for (int c = l0; c < q - 1; ++c) w.R()[l + c * LD] = w.R()[l + (c + 1) * LD];
                w.R()[l + (q - 1) * LD] = 0.0;
            }
            {
                int an = 0;
                double un = 0.0;
                if (l >= l0 && l < q) { an = w.act()[l + 1]; un = w.uu()[l + 1]; }
                NTM_WSYNC();
                if (l >= l0 && l < q) { w.act()[l] = an; w.uu()[l] = un; }
                if (l == 0) w.aflag()[dropped] = 0;
            }
            NTM_WSYNC();
            for (int j = l0; j < q - 1; ++j) {
                double a = w.R()[j + j * LD], bq = w.R()[(j + 1) + j * LD];
                double hh = hypot(a, bq);
                double cc = 1.0, ss = 0.0;
                if (hh != 0.0) { cc = a / hh; ss = bq / hh; }
                NTM_WSYNC();
                if (l >= j && l < q - 1) {
                    double r1 = w.R()[j + l * LD], r2 = w.R()[(j + 1) + l * LD];
                    w.R()[j + l * LD] = cc * r1 + ss * r2;
                    w.R()[(j + 1) + l * LD] = (l == j) ? 0.0 : (-ss * r1 + cc * r2);
                }
                if (l < N) {
                    double j1 = w.J()[l * LDJ + j], j2 = w.J()[l * LDJ + j + 1];
                    w.J()[l * LDJ + j] = cc * j1 + ss * j2;
                    w.J()[l * LDJ + j + 1] = -ss * j1 + cc * j2;
                }
                NTM_WSYNC();
            }
            --q;
        }
    }
}

// ---------------------------------------------------------------------------
// Exact re-solve on GI's final active set (oracle: polish_active_set).
//   Rows with a single non-zero fix their variable exactly (U_j = b/Lin_j);
//   the other active rows S are equality constraints on the free variables:
//   masked Cholesky of G~ (fixed rows/cols -> identity), Schur complement
//   K = E G~_FF^{-1} E', then V_F.  Accepted only if the KKT certificate
//   holds; otherwise w.U() keeps GI's solution.  Pre: w.V() = GI solution.
//   Writes w.U() (unscaled U).  G~ comes from Gamma (gram, structured rows) or
//   from Gsave (a copy taken before the GI factorisation, dense rows).
// ---------------------------------------------------------------------------
template <int P, class Rows>
__device__ bool polish_phase(const Prob& pb, const WS& w, const Rows* rows, int q, int l,
                             const double* Gsave, bool g_in_R, bool verify_only, int* ns_out) {
    const int N = w.N, LD = w.LDJ, LDJ = w.LDJ;
    const double Vgi = (l < N) ? w.V()[l] : 0.0;
    // --- classify active rows ---
    if (l < N) w.fx()[l] = 0;
    NTM_WSYNC();
    int isgen = 0, fixj = -1;
    double ufix = 0.0;
    int id = -1;
    if (l < q) {
        id = w.act()[l];
        int nnz = 0;
        for (int j = 0; j < N; ++j) if (rows->lin(w, id, j) != 0.0) { ++nnz; fixj = j; }
        if (nnz == 1) ufix = rows->bval(w, id) / rows->lin(w, id, fixj);
        else isgen = 1;
    }
    double nfix = 0.0;   // GI normal entry of the single-entry row (for its multiplier)
    if (l < q && !isgen) nfix = -((rows->lin(w, id, fixj) * w.D()[fixj]) / rows->rnorm(w, id));
    const unsigned long long gmask = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << ((threadIdx.x & 63) & ~(P - 1)));
    const unsigned long long bal = __ballot(isgen) & gmask;
    const int nS = __popcll(bal);
    const int spos = __popcll(bal & ((1ull << (threadIdx.x & 63)) - 1ull));
    if (l < q) {
        if (isgen) w.sidx()[spos] = id;
        else { w.fx()[fixj] = 1; w.Uf()[fixj] = ufix; w.hv()[fixj] = nfix; }
    }
    NTM_WSYNC();
    const bool fixed = (l < N) && w.fx()[l];
    const double vb = fixed ? w.Uf()[l] / w.D()[l] : 0.0;
    if (l < N) w.Vb()[l] = vb;
    if (ns_out) *ns_out = nS;
    // --- G~ again (bit-identical to the GI's copy), g = F~ + G~_{:,B} V_B ---
    if (g_in_R) {
        // candidate verification: G~ is still intact in w.R()
    } else if (Gsave) {
        if (l < N) for (int j = 0; j <= l; ++j) w.R()[l + j * LD] = Gsave[l + j * LD];
    } else {
        gram_rows<P>(pb, w, w.R(), l);
        NTM_WSYNC();
        (void)scale_gram<P>(w, w.R(), l);
    }
    NTM_WSYNC();
    double gl = 0.0;
    if (l < N) {
        gl = w.F()[l];
        for (int j = 0; j < N; ++j)
            if (w.fx()[j]) gl += ((j <= l) ? w.R()[l + j * LD] : w.R()[j + l * LD]) * w.Vb()[j];
        if (fixed) gl = 0.0;
    }
    NTM_WSYNC();
    if (l < N) {   // mask fixed rows/cols to identity (row l, columns <= l)
        for (int j = 0; j <= l; ++j)
            if (fixed || w.fx()[j]) w.R()[l + j * LD] = (j == l) ? 1.0 : 0.0;
    }
    NTM_WSYNC();
    bool ok = chol_inplace<P>(w.R(), N, LD, l);
    double vfin = 0.0;
    if (ok) {
        double wl = fwd_lanes<P>(w.R(), N, LD, gl, l);      // w = L^{-1} g
        double tl = -wl;
        if (nS > 0) {
            // E' into Y (= w.J(), row-major N x nS), h_s
            if (l < N) {
                for (int s = 0; s < nS; ++s) {
                    int rid = w.sidx()[s];
                    double nj = -((rows->lin(w, rid, l) * w.D()[l]) / rows->rnorm(w, rid));
                    w.J()[l * LDJ + s] = fixed ? 0.0 : nj;
                }
            }
            double hs = 0.0;
            if (l < nS) {
                int rid = w.sidx()[l];
                double rn = rows->rnorm(w, rid);
                hs = -(rows->bval(w, rid) / rn);
                for (int j = 0; j < N; ++j)
                    if (w.fx()[j]) hs -= (-((rows->lin(w, rid, j) * w.D()[j]) / rn)) * w.Vb()[j];
            }
            if (l < N) w.d()[l] = wl;
            NTM_WSYNC();
            // Y = L^{-1} E' : lane s solves column s in place
            if (l < nS) {
                for (int i = 0; i < N; ++i) {
                    double y = w.J()[i * LDJ + l];
                    for (int k = 0; k < i; ++k) y -= w.R()[i + k * LD] * w.J()[k * LDJ + l];
                    w.J()[i * LDJ + l] = y / w.R()[i + i * LD];
                }
            }
            NTM_WSYNC();
            // K = Y'Y (lower, col-major in w.M()); rhs = h + Y'w
            double rhs = 0.0;
            if (l < nS) {
                for (int c = 0; c <= l; ++c) {
                    double sK = 0.0;
                    for (int i = 0; i < N; ++i) sK += w.J()[i * LDJ + l] * w.J()[i * LDJ + c];
                    w.M()[l + c * LD] = sK;
                }
                rhs = hs;
                for (int i = 0; i < N; ++i) rhs += w.J()[i * LDJ + l] * w.d()[i];
            }
            NTM_WSYNC();
            ok = chol_inplace<P>(w.M(), nS, LD, l);
            if (ok) {
                double t1 = fwd_lanes<P>(w.M(), nS, LD, rhs, l);
                double mu = bwd_lanes<P>(w.M(), nS, LD, t1, l);
                if (l < nS) w.np()[l] = mu;
                NTM_WSYNC();
                if (l < N) {
                    double sY = 0.0;
                    for (int a = 0; a < nS; ++a) sY += w.J()[l * LDJ + a] * w.np()[a];
                    tl = sY - wl;
                }
            }
        }
        if (ok) {
            double vl = bwd_lanes<P>(w.R(), N, LD, tl, l);  // V_F = L^{-T} t
            vfin = fixed ? vb : vl;
        }
    }
    ok = gmaxi<P>(ok ? 0 : 1) == 0;
    if (ok) {
        // ---- KKT certificate ----
        if (l < N) w.V()[l] = vfin;
        NTM_WSYNC();
        double vmax = gmax<P>(l < N ? fabs(vfin) : 0.0);
        Pick vf = rows->template check<P>(w, vfin, l, true, fmax(1.0, vmax));
        ok = vf.p == 0;
        // gradient G~V + F~ (G~ itself is factored now)
        double res = 0.0;
        if (Gsave) {
            if (l < N) {
                res = w.F()[l];
                for (int j = 0; j < N; ++j)
                    res += ((j <= l) ? Gsave[l + j * LD] : Gsave[j + l * LD]) * w.V()[j];
            }
        } else {
            // through Gamma: y = Gamma (D V), grad_j = D_j 2 Gamma_j' Om y + F~_j
            for (int r = l; r < 2 * N; r += P) {
                double y = 0.0;
                for (int j = 0; j <= (r >> 1); ++j) y += w.Gt()[r + j * w.LDG] * (w.D()[j] * w.V()[j]);
                w.xp()[r] = y;              // scratch: xp is rewritten by the rollout
            }
            NTM_WSYNC();
            if (l < N) {
                double g2 = 0.0;
                for (int i = l; i < N; ++i) {
                    double y0 = w.xp()[2 * i], y1 = w.xp()[2 * i + 1];
                    double o0 = pb.Q[0] * y0 + pb.Q[1] * y1, o1 = pb.Q[2] * y0 + pb.Q[3] * y1;
                    g2 += w.Gt()[2 * i + l * w.LDG] * o0 + w.Gt()[2 * i + 1 + l * w.LDG] * o1;
                }
                res = w.D()[l] * (2 * g2) + w.F()[l];
            }
        }
        if (l < N) {
            for (int s = 0; s < nS; ++s) {
                int rid = w.sidx()[s];
                res -= w.np()[s] * (-((rows->lin(w, rid, l) * w.D()[l]) / rows->rnorm(w, rid)));
            }
        }
        // multipliers: mu_s (general rows) and res_j / n_j (fixed variables)
        double mval = 0.0;
        bool has = false;
        if (l < nS) { mval = w.np()[l]; has = true; }
        if (fixed) {
            double lam = res / w.hv()[l];
            mval = has ? fmin(mval, lam) : lam;
            has = true;
        }
        double mabs = gmax<P>(has ? fabs(mval) : 0.0);
        double mmin = -gmax<P>(has ? -mval : -kInf);
        ok = ok && !(mmin < -1e-9 * fmax(1.0, mabs));
    }
    if (verify_only && !ok) {
        if (l < N) w.V()[l] = Vgi;
        NTM_WSYNC();
        return false;
    }
    if (l < N) {
        double u;
        if (ok) u = fixed ? w.Uf()[l] : vfin * w.D()[l];
        else u = Vgi * w.D()[l];
        w.U()[l] = u;
        w.V()[l] = ok ? vfin : Vgi;
    }
    NTM_WSYNC();
    return ok;
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
        w.xp()[0] = y0;
        w.xp()[1] = y1;
        for (int i = 0; i < N; ++i) {
            double n0 = (w.a11()[i] * y0 + w.bb()[i] * w.U()[i]) + k.C1;
            double n1 = (w.a21()[i] * y0 + k.a22 * y1) + k.C2;
            y0 = n0;
            y1 = n1;
            w.xp()[2 * i + 2] = y0;
            w.xp()[2 * i + 3] = y1;
        }
    }
    NTM_WSYNC();
    double dsum = 0.0;
    if (l < N) {
        double r1, r2, r3;
        rho_eval(k, w.xp()[2 * l], w.xp()[2 * l + 1], r1, r2, r3);
        w.rho()[3 * l] = r1;
        w.rho()[3 * l + 1] = r2;
        w.rho()[3 * l + 2] = r3;
        double u = w.U()[l];
        dsum = fabs(w.Uold()[l] - u);
        w.Uold()[l] = u;
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
// one inner iteration's QP: build -> scale -> GI -> polish -> w.U()
// ---------------------------------------------------------------------------
template <int P>
__device__ int qp_phase(const Prob& pb, const WS& w, double x0, double x1, int l, int* qp_iters,
                        int* q_out, int* ns_out, int slot) {
    const int N = w.N;
    lift_phase<P>(pb, w, l);
    free_response<P>(w, x0, x1, l);
    cost_phase<P>(pb, w, l);
    const bool full = pb.mode == NTM_MODE_FULL;
    int flag, q = 0, ns = 0;
    *qp_iters = 0;
    StructRows rows(pb);
    int* cand = w.cand() + slot * (N + 1);
    if (!scale_phase<P>(w, l, full)) {
        flag = NTM_EXIT_NONFINITE;
    } else {
        const int nrows = (pb.mode == NTM_MODE_NONE) ? 0 : rows.rows();
        if (pb.mode != NTM_MODE_NONE) {
            for (int i = l; i < nrows; i += P) w.aflag()[i] = 0;
            NTM_WSYNC();
        }
        if (pb.mode != NTM_MODE_NONE && !rows.template feasible_const<P>(w, x0, x1, l)) {
            flag = NTM_EXIT_INFEASIBLE;
        } else {
            bool done = false;
            // warm start: the LPV loop alternates between two QPs (a 2-cycle),
            // so the active set of iteration it-2 is tried first; it is taken
            // only if the exact active-set solve passes the KKT certificate
            // (the optimum of this strictly convex QP is unique).
            const int cq = cand[N];
            if (cq >= 0) {
                if (l < cq) w.act()[l] = cand[l];
                NTM_WSYNC();
                if (polish_phase<P, StructRows>(pb, w, &rows, cq, l, nullptr, true, true, &ns)) {
                    flag = NTM_EXIT_OPTIMAL;
                    q = cq;
                    done = true;
                } else {
                    gram_rows<P>(pb, w, w.R(), l);    // the verification factored w.R()
                    NTM_WSYNC();
                    (void)scale_gram<P>(w, w.R(), l);
                    NTM_WSYNC();
                }
            }
            if (!done) {
                flag = gi_solve<P, StructRows>(w, pb.mode == NTM_MODE_NONE ? nullptr : &rows, nrows, l,
                                               qp_iters, &q);
                if (flag == NTM_EXIT_OPTIMAL)
                    (void)polish_phase<P, StructRows>(pb, w, &rows, q, l, nullptr, false, false, &ns);
            }
        }
    }
    if (flag != NTM_EXIT_OPTIMAL) {
        if (l < N) w.U()[l] = (flag == NTM_EXIT_MAXITER) ? w.V()[l] * w.D()[l] : 0.0;
        if (l == 0) cand[N] = -1;
    } else {
        if (l < q) cand[l] = w.act()[l];
        if (l == 0) cand[N] = q;
    }
    NTM_WSYNC();
    if (q_out) *q_out = q;
    if (ns_out) *ns_out = ns;
    return flag;
}

}  // namespace ntm
