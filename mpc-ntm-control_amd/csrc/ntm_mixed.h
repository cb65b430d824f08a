// ntm_mixed.h — the fp32 leg of BASELINE config 5 ("fp32 vs fp64 tolerance
// sweep"): a Goldfarb-Idnani dual active-set solve of the
// quadprog-level QP (NTM_MPC_Sim.m:97) carried out entirely in fp32 on
// fp32-rounded QP data (G, F, Lin, b each rounded to fp32 on load; Jacobi
// scaling, row norms, Cholesky, J = L^-T, R, directions, step lengths, the
// Householder adds and Givens drops all in fp32).  Its final active set is then
// refined in fp64: the exact re-solve + KKT certificate of the fp64 path
// (polish_phase), with the fp64 Goldfarb-Idnani solve as the fallback when the
// fp32 active set does not certify.  The fp64 product path never calls this.
//
// One scenario per 64-lane wave; lane l owns variable l (N <= 64).  Group
// reductions use __shfl_xor butterflies: every pairing is symmetric, so each
// lane ends with the bit-identical value and control flow stays uniform.
#pragma once
#include "ntm_device.h"

namespace ntm {

template <int P>
__device__ __forceinline__ float fsum(float v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, P);
    return v;
}
template <int P>
__device__ __forceinline__ int ior_g(int v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v |= __shfl_xor(v, o, P);
    return v;
}
template <int P>
__device__ __forceinline__ float fmaxg(float v) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, P));
    return v;
}
// argmin of (v, id), ties to the smaller id; identical in every lane
template <int P>
__device__ __forceinline__ void fargmin(float& v, int& id) {
#pragma unroll
    for (int o = P / 2; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, P);
        const int oid = __shfl_xor(id, o, P);
        if (ov < v || (ov == v && oid < id)) { v = ov; id = oid; }
    }
}

// fp32 workspace (LDS), all arrays N-strided row-major
struct GI32 {
    float *G, *J, *R;                 // N x N each: scaled Hessian (L after Cholesky), J, R (upper)
    float *D, *F, *V, *U, *np, *d, *z, *r, *u, *h;   // N (u: N + 1)
    float* rn;                        // m row norms (0: constant row)
    int* act;                         // N + 1 active row ids
    unsigned char* af;                // m active flags
    int N, m;
    __host__ __device__ static size_t bytes(int N, int m) {
        size_t b = 3 * (size_t)N * N * 4 + (10 * (size_t)N + 1) * 4 + (size_t)m * 4 + (size_t)(N + 1) * 4 + m;
        return (b + 15) & ~(size_t)15;
    }
    __device__ void carve(char* base, int N_, int m_) {
        N = N_;
        m = m_;
        float* f = reinterpret_cast<float*>(base);
        G = f; f += N * N;
        J = f; f += N * N;
        R = f; f += N * N;
        D = f; f += N;
        F = f; f += N;
        V = f; f += N;
        U = f; f += N;
        np = f; f += N;
        d = f; f += N;
        z = f; f += N;
        r = f; f += N;
        h = f; f += N;
        u = f; f += N + 1;
        rn = f; f += m;
        act = reinterpret_cast<int*>(f);
        af = reinterpret_cast<unsigned char*>(act + N + 1);
    }
};

// Dense rows of the scenario in global memory (scenario-major, as ntm_qp_device)
struct Dense32 {
    const double* Lin;
    const double* b;
    int64_t s;
    int N, m;
    __device__ __forceinline__ float lin(int i, int j) const {
        return (float)Lin[s * ((int64_t)m * N) + i + (int64_t)j * m];
    }
    __device__ __forceinline__ float bv(int i) const { return (float)b[s * m + i]; }
};

// fp32 Goldfarb-Idnani on min 1/2 U'GU + F'U s.t. Lin U <= b (fp32-rounded data).
// Returns a quadprog exit flag; the active set in g.act[0..*q_out), U in g.U.
template <int P>
__device__ int gi32_solve(GI32& g, const double* G64, const double* F64, const Dense32& rows, int64_t s, int l,
                          int* q_out, int* iters_out) {
    const int N = g.N, m = g.m;
    *q_out = 0;
    *iters_out = 0;
    // --- fp32 data and Jacobi scaling U = D V (diag(D G D) = 1) ---
    if (l < N) {
        const float gll = (float)G64[s * (N * N) + l + l * N];
        g.D[l] = gll > 0.0f ? 1.0f / sqrtf(gll) : 1.0f;
    }
    NTM_WSYNC();
    int bad = 0;
    if (l < N) {
        for (int k = 0; k < N; ++k) {
            const float v = (float)G64[s * (N * N) + l + k * N] * g.D[l] * g.D[k];
            bad |= !isfinite(v);
            g.G[l * N + k] = v;
        }
        const float f = (float)F64[s * N + l] * g.D[l];
        bad |= !isfinite(f);
        g.F[l] = f;
    }
    for (int i = l; i < m; i += P) {
        float ss = 0.0f;
        for (int j = 0; j < N; ++j) {
            const float v = rows.lin(i, j) * g.D[j];
            ss += v * v;
        }
        bad |= !isfinite(ss) || !isfinite(rows.bv(i));
        g.rn[i] = ss > 0.0f ? sqrtf(ss) : 0.0f;
        if (!(ss > 0.0f) && rows.bv(i) < -1e-6f) bad |= 2;          // violated constant row (D15)
        g.af[i] = 0;
    }
    NTM_WSYNC();
    bad = ior_g<P>(bad);
    if (bad & 1) return NTM_EXIT_NONFINITE;
    if (bad & 2) return NTM_EXIT_INFEASIBLE;
    // --- Cholesky G~ = L L' (lower, in place, left-looking by columns) ---
    for (int k = 0; k < N; ++k) {
        float sl = 0.0f;
        if (l >= k && l < N) {
            sl = g.G[l * N + k];
            for (int j = 0; j < k; ++j) sl -= g.G[l * N + j] * g.G[k * N + j];
        }
        const float dk = __shfl(sl, k, P);
        if (!(dk > 0.0f)) return NTM_EXIT_NONFINITE;
        const float rd = sqrtf(dk);
        if (l >= k && l < N) g.G[l * N + k] = (l == k) ? rd : sl / rd;
        NTM_WSYNC();
    }
    // --- J = L^-T: lane c solves L x = e_c (column c of L^-1 = row c of J) ---
    if (l < N) {
        for (int i = 0; i < N; ++i) {
            float x = 0.0f;
            if (i >= l) {
                x = (i == l) ? 1.0f : 0.0f;
                for (int j = l; j < i; ++j) x -= g.G[i * N + j] * g.J[l * N + j];
                x /= g.G[i * N + i];
            }
            g.J[l * N + i] = x;
        }
        for (int i = 0; i < N; ++i) g.R[l * N + i] = 0.0f;
    }
    NTM_WSYNC();
    // --- unconstrained V = -J J' F~ ---
    if (l < N) {
        float t = 0.0f;
        for (int j = 0; j < N; ++j) t += g.J[j * N + l] * g.F[j];
        g.d[l] = t;
    }
    NTM_WSYNC();
    if (l < N) {
        float v = 0.0f;
        for (int k = 0; k < N; ++k) v += g.J[l * N + k] * g.d[k];
        g.V[l] = -v;
        g.U[l] = g.D[l] * -v;
    }
    NTM_WSYNC();
    if (m == 0) return NTM_EXIT_OPTIMAL;
    const int max_iter = 10 * (N + m) + 50;
    int q = 0, it = 0;
    constexpr float kInfF = __builtin_huge_valf();
    while (it < max_iter) {
        // most violated inactive row: slack (b_i - Lin_i U) / rn_i (GI form n'V - bc)
        float best = kInfF, bbc = 0.0f;
        int bid = 0x7fffffff;
        const float vmax = fmaxg<P>(l < N ? fabsf(g.V[l]) : 0.0f);
        for (int i = l; i < m; i += P) {
            const float rn = g.rn[i];
            if (rn > 0.0f && !g.af[i]) {
                float lu = 0.0f;
                for (int j = 0; j < N; ++j) lu += rows.lin(i, j) * g.U[j];
                const float bc = -rows.bv(i) / rn;
                const float sl = (rows.bv(i) - lu) / rn;
                if (sl < -1e-6f * fmaxf(1.0f, fmaxf(vmax, fabsf(bc))) && (sl < best || (sl == best && i < bid))) {
                    best = sl;
                    bid = i;
                    bbc = bc;
                }
            }
        }
        const float bc_own = bbc;
        fargmin<P>(best, bid);
        if (!(best < kInfF)) break;                                  // no violated row: optimal
        const int p = bid;
        const float bcp = __shfl(bc_own, p % P, P);                  // the winner's bc (lane p mod P found it)
        const float rnp = g.rn[p];
        if (l < N) g.np[l] = -(rows.lin(p, l) * g.D[l]) / rnp;
        NTM_WSYNC();
        float up = 0.0f;                                            // multiplier of p while it is added
        bool added = false;
        while (!added && it < max_iter) {
            ++it;
            // d = J' n_p ; z = J2 d2 ; r = R^-1 d1
            if (l < N) {
                float dl = 0.0f;
                for (int j = 0; j < N; ++j) dl += g.J[j * N + l] * g.np[j];
                g.d[l] = dl;
            }
            NTM_WSYNC();
            float zl = 0.0f;
            if (l < N) {
                for (int k = q; k < N; ++k) zl += g.J[l * N + k] * g.d[k];
                g.z[l] = zl;
            }
            const float d2n = fsum<P>((l >= q && l < N) ? g.d[l] * g.d[l] : 0.0f);
            if (l == 0) {
                for (int a = q - 1; a >= 0; --a) {
                    float x = g.d[a];
                    for (int c = a + 1; c < q; ++c) x -= g.R[a * N + c] * g.r[c];
                    g.r[a] = x / g.R[a * N + a];
                }
            }
            NTM_WSYNC();
            // step lengths
            float t1 = kInfF;
            int k1 = 0x7fffffff;
            if (l < q && g.r[l] > 0.0f) { t1 = g.u[l] / g.r[l]; k1 = l; }
            fargmin<P>(t1, k1);
            const float nv = fsum<P>(l < N ? g.np[l] * g.V[l] : 0.0f);
            const float sp = nv - bcp;                                // n'V - bc < 0 while violated
            const float dnorm = fsum<P>(l < N ? g.d[l] * g.d[l] : 0.0f);
            const float t2 = (d2n > 1e-10f * dnorm) ? -sp / d2n : kInfF;
            if (!(t1 < kInfF) && !(t2 < kInfF)) { *q_out = q; *iters_out = it; return NTM_EXIT_INFEASIBLE; }
            const float t = fminf(t1, t2);
            if (t2 < kInfF && l < N) {                                // primal + dual step
                g.V[l] += t * zl;
                g.U[l] = g.D[l] * g.V[l];
            }
            if (l < q) g.u[l] -= t * g.r[l];
            up += t;
            NTM_WSYNC();
            if (t2 <= t1) {
                // add p: Householder on d2 (zeroes d_{q+1..N-1}); J2 <- J2 H; R(:, q) = [d1; alpha]
                const float sig = sqrtf(d2n);
                const float dq = g.d[q];
                const float alpha = dq > 0.0f ? -sig : sig;
                if (l >= q && l < N) g.h[l] = (l == q) ? dq - alpha : g.d[l];
                NTM_WSYNC();
                const float beta = fsum<P>((l >= q && l < N) ? g.h[l] * g.h[l] : 0.0f);
                if (beta > 0.0f && l < N) {
                    float w = 0.0f;
                    for (int k = q; k < N; ++k) w += g.J[l * N + k] * g.h[k];
                    const float f = 2.0f * w / beta;
                    for (int k = q; k < N; ++k) g.J[l * N + k] -= f * g.h[k];
                }
                if (l < q) g.R[l * N + q] = g.d[l];
                if (l == q) g.R[q * N + q] = alpha;
                if (l == 0) {
                    g.act[q] = p;
                    g.u[q] = up;
                    g.af[p] = 1;
                }
                NTM_WSYNC();
                ++q;
                added = true;
            } else {
                // drop row k1: R loses column k1, Givens rotations restore the triangle
                const int k = k1;
                if (l == 0) g.af[g.act[k]] = 0;
                NTM_WSYNC();
                const int an = (l + 1 < q) ? g.act[l + 1] : 0;
                const float un = (l + 1 < q) ? g.u[l + 1] : 0.0f;
                NTM_WSYNC();
                if (l >= k && l + 1 < q) { g.act[l] = an; g.u[l] = un; }
                // shift R's columns k+1..q-1 left (lane = row)
                if (l < N)
                    for (int c = k; c + 1 < q; ++c) g.R[l * N + c] = g.R[l * N + c + 1];
                if (l < N) g.R[l * N + (q - 1)] = 0.0f;
                NTM_WSYNC();
                for (int j = k; j + 1 < q; ++j) {
                    const float a = g.R[j * N + j], bq = g.R[(j + 1) * N + j];
                    const float hh = sqrtf(a * a + bq * bq);
                    const float cc = hh > 0.0f ? a / hh : 1.0f, ssn = hh > 0.0f ? bq / hh : 0.0f;
                    if (l >= j && l < N) {                           // rows j, j+1 of R, column l
                        const float r1 = g.R[j * N + l], r2 = g.R[(j + 1) * N + l];
                        g.R[j * N + l] = cc * r1 + ssn * r2;
                        g.R[(j + 1) * N + l] = (l == j) ? 0.0f : -ssn * r1 + cc * r2;
                    }
                    if (l < N) {                                     // columns j, j+1 of J, row l
                        const float j1 = g.J[l * N + j], j2 = g.J[l * N + j + 1];
                        g.J[l * N + j] = cc * j1 + ssn * j2;
                        g.J[l * N + j + 1] = -ssn * j1 + cc * j2;
                    }
                    NTM_WSYNC();
                }
                --q;
            }
        }
    }
    *q_out = q;
    *iters_out = it;
    return it >= max_iter ? NTM_EXIT_MAXITER : NTM_EXIT_OPTIMAL;
}

}  // namespace ntm
