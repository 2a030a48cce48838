// ba_chol.hip -- dense reduced-camera solve on gfx950: blocked right-looking
// tile Cholesky with fp64 MFMA (v_mfma_f64_16x16x4_f64) + triangular solves.
//
// Replaces da = pinv(S) * e_ (toolbox/bundle/bundle_euclid.m:193).  S is
// symmetric positive definite once its exactly-zero rows (fixed parameters,
// App. A Q2/Q8) are given a unit diagonal (k_assemble_tiles), and on that matrix
// pinv and the Cholesky solve agree to conditioning-limited rounding.  A
// non-positive pivot sets status[0]; the host then takes da = pinv(S) e_
// (rocSOLVER dsyevd, ba_solver.cpp pinv_fallback), as bundle_euclid.m:193 does.
//
// Storage: S column major, leading dimension lds (multiple of NB = 64), lower
// triangle.  Tile envelope: tile row i of S (hence of L: the profile is
// preserved by Cholesky) is zero left of tile column tfirst[i]; every kernel
// below visits only tiles inside the envelope, which is exact (the skipped
// tiles are zero and stay zero).  dense_solve = 1 visits every lower tile.
//
// Per tile column k (one launch, k_factor_step):
//   WG 0     : applies column k-1's update to A_kk, factors L_kk, forms
//              L_kk^-1 and y_k = L_kk^-1 r_k (forward solve folded in);
//   WG b > 0 : applies column k-1's update to A_ik, redoes A_kk's update and
//              factorisation in LDS and forms the panel tile L_ik = A_ik L_kk^-T
//              (MFMA), r_i -= L_ik y_k;
//   the rest : column k-1's trailing update A_ij -= L_i,k-1 L_j,k-1^T of the
//              envelope pairs below row k (MFMA)
// then the backward solve x_k = L_kk^-T z_k, z_j -= L_kj^T x_k (one launch,
// k_backward_all, or per column k_backward).
//
// Solvers on top of the tiles (ba_chol_setup picks one): block cyclic
// reduction when S is tile-tridiagonal (k_cr32_fused on camera-aligned 30-row
// tiles); else the envelope Cholesky, on a nested-dissection camera order
// (arcs side by side in k_factor_multi, separator SYRK k_sep_update /
// k_sep_reduce, then the separator) when that shortens the chain of columns;
// the sequential k_chol_seq in parity mode.
#include "ba_internal.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <cstdio>
#include <utility>
#include <climits>
#include <cstdlib>
#include <vector>

#define NB 64
#define LP 66  // LDS row pitch (doubles): conflict-free 16x4 MFMA operand reads

typedef double d4 __attribute__((ext_vector_type(4)));

// S tile (ti, tj) -> LDS row-major T[r][c] (256 threads).  Thread (r = tid&63,
// c0 = tid>>6) moves column c0 + 4u, u = 0..15: each wave reads whole 512-B
// columns (coalesced) and all 16 loads are in flight before the LDS writes.
__device__ __forceinline__ void load_tile(const double *__restrict__ S, long long lds, int ti,
                                          int tj, double *T)
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = base[r + lds * (c0 + 4 * u)];
#pragma unroll
    for (int u = 0; u < 16; u++) T[r * LP + c0 + 4 * u] = v[u];
}

// S tile (ti, tj) transposed -> LDS T[c][r] = tile[r][c] (LDS writes contiguous in r)
__device__ __forceinline__ void load_tile_t(const double *__restrict__ S, long long lds, int ti,
                                            int tj, double *T)
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = base[r + lds * (c0 + 4 * u)];
#pragma unroll
    for (int u = 0; u < 16; u++) T[(c0 + 4 * u) * LP + r] = v[u];
}

// split forms of load_tile / load_tile_t: fetch to registers, then put, so
// that several tiles' loads can be in flight together
__device__ __forceinline__ void fetch_tile(const double *__restrict__ S, long long lds, int ti,
                                           int tj, double v[16])
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = base[r + lds * (c0 + 4 * u)];
}

__device__ __forceinline__ void put_tile(double *T, const double v[16], bool transposed)
{
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        if (transposed)
            T[(c0 + 4 * u) * LP + r] = v[u];
        else
            T[r * LP + c0 + 4 * u] = v[u];
    }
}

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned gu32_t;

template <bool SC> __device__ __forceinline__ double ldg(const double *p)
{
    if constexpr (SC)
        return __builtin_bit_cast(
            double, __hip_atomic_load((gu64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    else
        return *p;
}

template <bool SC> __device__ __forceinline__ void stg(double *p, double v)
{
    if constexpr (SC)
        __hip_atomic_store((gu64_t *)p, __builtin_bit_cast(unsigned long long, v),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// fetch_tile / store_tile with device-coherent (sc1) accesses: tiles handed
// between the envelope runner and the column launches running beside it
__device__ __forceinline__ void fetch_tile_sc(const double *S, long long lds, int ti, int tj,
                                              double v[16])
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = ldg<true>(base + r + lds * (c0 + 4 * u));
}

__device__ __forceinline__ void store_tile_sc(double *S, long long lds, int ti, int tj,
                                              const double *T)
{
    double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = T[r * LP + c0 + 4 * u];
#pragma unroll
    for (int u = 0; u < 16; u++) stg<true>(base + r + lds * (c0 + 4 * u), v[u]);
}

// LDS T[r][c] -> row-major 64x64 dst[r*64 + c]
__device__ __forceinline__ void store_rowmajor(double *__restrict__ dst, const double *T)
{
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = T[(r0 + 4 * u) * LP + c];
#pragma unroll
    for (int u = 0; u < 16; u++) dst[(r0 + 4 * u) * NB + c] = v[u];
}

// row-major 64x64 (src[r*64 + c]) -> LDS T[r][c], loads batched as above
__device__ __forceinline__ void load_rowmajor(const double *__restrict__ src, double *T)
{
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = src[(r0 + 4 * u) * NB + c];
#pragma unroll
    for (int u = 0; u < 16; u++) T[(r0 + 4 * u) * LP + c] = v[u];
}

__device__ __forceinline__ void store_tile(double *__restrict__ S, long long lds, int ti, int tj,
                                           const double *T)
{
    double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = threadIdx.x & 63, c0 = threadIdx.x >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = T[r * LP + c0 + 4 * u];
#pragma unroll
    for (int u = 0; u < 16; u++) base[r + lds * (c0 + 4 * u)] = v[u];
}

// acc = As[r][:] . Bs[c][:] over K = 64 for the 64x64 tile of a 256-thread WG.
// Wave w owns rows 32*(w>>1) .. +31, cols 32*(w&1) .. +31 as 2x2 MFMA tiles.
// f64 16x16x4 operand map: A lane l -> A[l&15][l>>4], B lane l -> B[l>>4][l&15];
// result register q of lane l -> (row (l>>4) + 4q, col l&15).
__device__ __forceinline__ void mfma_64x64_acc(const double *As, const double *Bs, d4 acc[2][2])
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
    for (int s = 0; s < NB / 4; s++) {
        const int kk = 4 * s + lk;
        const double a0 = As[(r0 + li) * LP + kk];
        const double a1 = As[(r0 + 16 + li) * LP + kk];
        const double b0 = Bs[(c0 + li) * LP + kk];
        const double b1 = Bs[(c0 + 16 + li) * LP + kk];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
}

__device__ __forceinline__ void mfma_64x64(const double *As, const double *Bs, d4 acc[2][2])
{
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
    mfma_64x64_acc(As, Bs, acc);
}

// acc = A B^T over K = 64 for A = S tile (ia, kc), B = S tile (jb, kc), the
// operands read straight from S (column-major, L2) in the 16x16x4 operand
// layout instead of from LDS: the same MFMA chain as mfma_64x64 on the
// loaded tiles, bit for bit, without their 64 KB of LDS.
template <bool SCB = false>
__device__ __forceinline__ void mfma_64x64_glb(const double *__restrict__ S, long long lds,
                                               int ia, int jb, int kc, d4 acc[2][2])
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    const int li = lane & 15, lk = lane >> 4;
    const double *A = S + (long long)NB * ia + lds * (long long)NB * kc;
    const double *B = S + (long long)NB * jb + lds * (long long)NB * kc;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; h++) {   // K in two halves of operand loads
        double a0[8], a1[8], b0[8], b1[8];
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const long long kk = lds * (4 * (8 * h + s) + lk);
            a0[s] = A[r0 + li + kk];
            a1[s] = A[r0 + 16 + li + kk];
            b0[s] = ldg<SCB>(B + c0 + li + kk);
            b1[s] = ldg<SCB>(B + c0 + 16 + li + kk);
        }
#pragma unroll
        for (int s = 0; s < 8; s++) {
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s], b0[s], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s], b1[s], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], b0[s], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], b1[s], acc[1][1], 0, 0, 0);
        }
    }
}

// write acc (scale * acc + (add ? T : 0)) into LDS tile T in MFMA layout
__device__ __forceinline__ void acc_to_lds(const d4 acc[2][2], double *T, double scale, bool add)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = r0 + 16 * x + (lane >> 4) + 4 * q, c = c0 + 16 * y + (lane & 15);
                const double v = scale * acc[x][y][q];
                T[r * LP + c] = add ? T[r * LP + c] + v : v;
            }
}

// ---- 16x16 MFMA helpers on LDS row-major tiles (pitch LP), one wave each ----
// nt: acc[r][c] += sum_t A[ra+r][ka+t] * Bt[cb+c][kb+t]   (B given transposed)
// nn: acc[r][c] += sum_t A[ra+r][ka+t] * Bn[kb+t][cb+c]
__device__ __forceinline__ d4 mfma16_nt(const double *A, int ra, int ka, const double *Bt, int cb,
                                        int kb, d4 acc)
{
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 4; s++)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(ra + li) * LP + ka + 4 * s + lk],
                                                   Bt[(cb + li) * LP + kb + 4 * s + lk], acc,
                                                   0, 0, 0);
    return acc;
}

__device__ __forceinline__ d4 mfma16_nn(const double *A, int ra, int ka, const double *Bn, int kb,
                                        int cb, d4 acc)
{
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 4; s++)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(ra + li) * LP + ka + 4 * s + lk],
                                                   Bn[(kb + 4 * s + lk) * LP + cb + li], acc,
                                                   0, 0, 0);
    return acc;
}

// T[r0 + row][c0 + col] = scale * acc (+ T if add): 16x16 result layout
__device__ __forceinline__ void put16(double *T, int r0, int c0, d4 acc, double scale, bool add)
{
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        double *p = T + (r0 + lk + 4 * q) * LP + c0 + li;
        *p = add ? *p + scale * acc[q] : scale * acc[q];
    }
}

// out = scale * M v for a 64x64 LDS tile (row-major, pitch LP) and a 64-vector
// in LDS, by all 256 threads: thread (row, quarter) sums 16 columns, the four
// quarters are added in fixed order.  Result to LDS out[] (if non-null) and to
// reg[0] of threads 0..63 (if non-null).  Ends with a barrier.
__device__ __forceinline__ void gemv64(const double *M, const double *v, double (*part)[NB],
                                       double *out, double scale, double *reg = nullptr)
{
    const int tid = threadIdx.x, row = tid & 63, qq = tid >> 6;
    double s = 0.0;
#pragma unroll
    for (int c = 16 * qq; c < 16 * qq + 16; c++) s = fma(M[row * LP + c], v[c], s);
    part[qq][row] = s;
    __syncthreads();
    if (tid < NB) {
        const double t = scale * (((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid]);
        if (out) out[tid] = t;
        if (reg) reg[0] = t;
    }
    __syncthreads();
}

// out[c] = scale * sum_r M[r][c] v[r] (M^T v), same thread split and order as gemv64
__device__ __forceinline__ void gemv64_t(const double *M, const double *v, double (*part)[NB],
                                         double *out, double scale)
{
    const int tid = threadIdx.x, c = tid & 63, qq = tid >> 6;
    double s = 0.0;
#pragma unroll
    for (int r = 16 * qq; r < 16 * qq + 16; r++) s = fma(M[r * LP + c], v[r], s);
    part[qq][c] = s;
    __syncthreads();
    if (tid < NB) out[tid] = scale * (((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid]);
    __syncthreads();
}

static __device__ __forceinline__ double rdlane(double v, int l)
{
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffLL), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// lane q's value to every lane of its 16-lane row (DPP row_newbcast, one
// v_mov_b64_dpp; no SGPR round trip).  q must fold to a constant.
template <int Q> __device__ __forceinline__ double rowbcast_c(double v)
{
    const long long u = __builtin_bit_cast(long long, v);
    const long long r = __builtin_amdgcn_mov_dpp(u, 0x150 + Q, 0xf, 0xf, true);
    return __builtin_bit_cast(double, r);
}

static __device__ __forceinline__ double rowbcast(double v, int q)
{
    switch (q) {
    case 0: return rowbcast_c<0>(v);
    case 1: return rowbcast_c<1>(v);
    case 2: return rowbcast_c<2>(v);
    case 3: return rowbcast_c<3>(v);
    case 4: return rowbcast_c<4>(v);
    case 5: return rowbcast_c<5>(v);
    case 6: return rowbcast_c<6>(v);
    case 7: return rowbcast_c<7>(v);
    case 8: return rowbcast_c<8>(v);
    case 9: return rowbcast_c<9>(v);
    case 10: return rowbcast_c<10>(v);
    case 11: return rowbcast_c<11>(v);
    case 12: return rowbcast_c<12>(v);
    case 13: return rowbcast_c<13>(v);
    case 14: return rowbcast_c<14>(v);
    default: return rowbcast_c<15>(v);
    }
}

// One wave: Cholesky of the 16x16 diagonal block at (o, o) of As and its
// inverse (lane r keeps row r of L and column r of L^-1 in registers; column
// broadcasts by DPP, pivots by readlane).  L (zero upper) -> As, L^-1 (zero
// upper) -> Bs.  The inverse's right-looking substitution (x_t /= L_tt,
// x_q -= L_qt x_t) runs inside the factor loop: its step t needs only column t
// of L, final at iteration t, and shares that column's DPP broadcasts L_qt with
// the rank-1 update -- its FMAs fill the latency of the next pivot's rsqrt
// chain instead of forming a second dependent loop (same operations in the
// same order as a separate loop: bit-identical).
__device__ __forceinline__ bool wave_factor16(double *As, double *Bs, int o)
{
    const int r = threadIdx.x & 63;
    double d[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) d[c] = (r < 16) ? As[(o + r) * LP + o + c] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) x[q] = (q == r) ? 1.0 : 0.0;
    // 1/sqrt of a pivot: hardware estimate + two Newton steps (full fp64).  No
    // test on the chain: a pivot <= 0 (or NaN) makes its diagonal entry
    // piv * rsq(piv) NaN, which the check after the loop finds
    auto rsq = [&](double piv) {
        double y = __builtin_amdgcn_rsq(piv);
        const double hp = 0.5 * piv;
        y = y * fma(-hp * y, y, 1.5);
        y = y * fma(-hp * y, y, 1.5);
        return y;
    };
    // pivots reach every lane of the row by a DPP broadcast (a VGPR: no
    // readlane -> SGPR -> VALU hazard wait on the chain)
    double y = rsq(rowbcast_c<0>(d[0]));
#pragma unroll
    for (int c = 0; c < 16; c++) {
        // Unpredicated: lane c's d[c] * y is its pivot times y, the diagonal
        // of L; lanes r < c scale / update only their upper part, which is
        // never broadcast (broadcasts read lanes q > c) and is zeroed at the
        // store below.
        d[c] = d[c] * y;
        x[c] = x[c] * y;
        // look-ahead: column c+1 first, so the next pivot's rsqrt chain can
        // overlap the rest of this column's rank-1 update
        if (c + 1 < 16) {
            const double b = rowbcast(d[c], c + 1);
            d[c + 1] = fma(-d[c], b, d[c + 1]);
            y = rsq(rowbcast(d[c + 1], c + 1));
            x[c + 1] = fma(-b, x[c], x[c + 1]);
        }
#pragma unroll
        for (int q = c + 2; q < 16; q++) {
            const double b = rowbcast(d[c], q);
            d[q] = fma(-d[c], b, d[q]);
            x[q] = fma(-b, x[c], x[q]);
        }
        // keep each column's inverse updates with its broadcasts: left alone,
        // the compiler sinks them below the loop and parks the 120 broadcasts
        // in AGPRs until then (an empty asm that "modifies" x pins them here)
#pragma unroll
        for (int q = c; q < 16; q++) asm volatile("" : "+v"(x[q]));
    }
    double dg = 1.0;   // lane r's diagonal entry L_rr = sqrt(pivot r)
#pragma unroll
    for (int c = 0; c < 16; c++)
        if (r == c) dg = d[c];
    const bool ok = __all(r >= 16 || (dg > 0.0 && dg < __builtin_inf()));
    if (r < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) As[(o + r) * LP + o + c] = (c <= r) ? d[c] : 0.0;
#pragma unroll
        for (int c = 0; c < 16; c++) Bs[(o + c) * LP + o + r] = x[c];
    }
    return ok;
}

// The 256-thread workgroup factors the 64x64 SPD tile in As (row-major, lower
// used) and inverts the factor, blocked by 16 (blocks 0..3).  Per block column
// k one wave factors the diagonal block (wave_factor16: L_kk and its inverse),
// the panel blocks L_ik = A_ik Dinv_kk^T follow on the matrix pipe, then the
// trailing blocks A_ij -= L_ik L_jk^T.  Look-ahead schedule: wave 0 updates
// the next diagonal block first and factors it at once, while the other waves
// finish the trailing blocks and form the off-diagonal blocks of L^-1,
//     Li_ij = -Li_ii sum_{t=j}^{i-1} L_it Li_tj,
// as soon as their inputs exist -- the critical path is the four diagonal
// factorisations plus three panel steps.  Every block is formed by exactly
// the operations of the plain right-looking order, so the result is the
// same bit for bit.  Writes L to the lower triangle of As (the upper
// triangle is zeroed only if zero_upper: the 16x16 blocks above the diagonal
// keep A otherwise) and L^-1 (zero upper) to Li.  Returns false on a
// non-positive pivot.  The caller synchronises after filling As; the result
// is visible after return.
__device__ __forceinline__ bool block_potrf_inv(double *As, double *Li, bool zero_upper = true)
{
    __shared__ double Xs[4][16 * LP];
    __shared__ __attribute__((aligned(16))) int bad;   // keeps the static LDS a
                                                       // multiple of 16 B (G17)
    const int tid = threadIdx.x, w = tid >> 6;
    // one trailing block (i, j) of block column k: A_ij -= L_ik L_jk^T
    auto trail = [&](int i, int j, int k) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nt(As, 16 * i, 16 * k, As, 16 * j, 16 * k, acc);
        put16(As, 16 * i, 16 * j, acc, -1.0, true);
    };
    // one panel block: L_ik = A_ik Dinv_kk^T
    auto panel = [&](int i, int k) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nt(As, 16 * i, 16 * k, Li, 16 * k, 16 * k, acc);
        put16(As, 16 * i, 16 * k, acc, 1.0, false);
    };
    // one off-diagonal block of the inverse, Li_ij (i > j), by wave w (> 0)
    auto inv = [&](int i, int j) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int t = j; t < i; t++) acc = mfma16_nn(As, 16 * i, 16 * t, Li, 16 * t, 16 * j, acc);
        put16(Xs[w], 0, 0, acc, 1.0, false);
        d4 acc2 = {0.0, 0.0, 0.0, 0.0};
        acc2 = mfma16_nn(Li, 16 * i, 16 * i, Xs[w], 0, 0, acc2);
        put16(Li, 16 * i, 16 * j, acc2, -1.0, false);
    };
    auto f16 = [&](int k) {
        if (!wave_factor16(As, Li, 16 * k) && (tid & 63) == 0) bad = 1;
    };
    // the six 16x16 blocks above the diagonal of L^-1 (everything else is
    // written below); ordered before their readers by the step barriers
    for (int q = tid; q < 6 * 256; q += blockDim.x) {
        const int b = q >> 8, e = q & 255;
        const int bi = b < 3 ? 0 : (b < 5 ? 1 : 2), bj = b < 3 ? b + 1 : (b < 5 ? b - 1 : 3);
        Li[(16 * bi + (e >> 4)) * LP + 16 * bj + (e & 15)] = 0.0;
    }
    if (tid == 0) bad = 0;   // same wave as the writer below: program order
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
        // A(k): wave 0 updates diagonal block k by column k-1 and factors it;
        // waves 1-3 apply column k-1 to the other trailing blocks
        if (w == 0) {
            if (k > 0) trail(k, k, k - 1);
            f16(k);
        } else if (k > 0) {
            int p = 0;
            for (int j = k; j < 4; j++)
                for (int i = j; i < 4; i++) {
                    if (i == k && j == k) continue;
                    if (1 + p % 3 == w) trail(i, j, k - 1);
                    p++;
                }
        }
        __syncthreads();
        // B(k): three tasks for waves 1-3 -- the panels of column k, then the
        // inverse blocks of block row k
        if (w >= 1) {
            const int t = w - 1;
            if (t < 3 - k)
                panel(k + 1 + t, k);
            else
                inv(k, t - (3 - k));
        }
        __syncthreads();
    }
    if (zero_upper) {
        for (int q = tid; q < NB * NB; q += blockDim.x) {   // zero the upper triangle of L
            const int r = q >> 6, c = q & 63;
            if (c > r) As[r * LP + c] = 0.0;
        }
        __syncthreads();
    }
    return bad == 0;
}

// ---------------------------------------------------------------------------
// One tile column k of the envelope Cholesky, with the trailing update of
// column k-1 folded in (one launch per column instead of two):
//   blockIdx 0        : A_kk -= L_{k,k-1} L_{k,k-1}^T (if column k-1 reaches
//                       row k), factor it, L_kk^-1, y_k = L_kk^-1 r_k
//   1 .. T            : panel tile i = pan[b-1]: A_ik -= L_{i,k-1} L_{k,k-1}^T,
//                       the same update + factorisation of A_kk in LDS
//                       (bit-identical), L_ik = A_ik L_kk^-T, r_i -= L_ik y_k
//   T+1 ..            : the rest of column k-1's trailing update,
//                       A_ij -= L_{i,k-1} L_{j,k-1}^T for envelope pairs of
//                       column k-1 with k < j <= i
// Every tile receives the same operations in the same order as the two-launch
// schedule (acc formed from zero, then A + (-1) acc): bit-identical results.
// pan / prev: the envelope rows below k / below k-1 (ascending), T / Tp their
// counts (Tp = 0 for k = 0).
// ---------------------------------------------------------------------------
#ifdef BA_STAMPS
// per tile column k: [0..3] workgroup 0 entry / factor start / factor end /
// exit, [4..7] the same for workgroup 1 (first panel tile), [8] the last exit
#define FS_MAX 4096
__device__ unsigned long long g_fst[FS_MAX][9];
extern "C" int vlgba_debug_fstamps(unsigned long long *out, int n)
{
    if (n > FS_MAX) n = FS_MAX;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fst), sizeof(unsigned long long) * 9 * n) ==
                   hipSuccess
               ? 0
               : -1;
}
#define FS_ST(q)                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0 && b <= 1 && k < FS_MAX)                                     \
            g_fst[k][4 * b + (q)] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
#define FS_END()                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0 && k < FS_MAX)                                               \
            atomicMax(&g_fst[k][8], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#else
#define FS_ST(q)
#define FS_END()
#endif

// sep0: the nested dissection's first separator row tile (INT_MAX: none):
// an arc column leaves the separator's rhs to k_sep_update (two arcs'
// columns run in the same launch) and its separator x separator trailing
// pairs, which the host does not launch (they end each pair enumeration).
// the 64 x 64 diagonal factor + inverse as two 32 x 32 factors (defined below)
__device__ __forceinline__ bool potrf64_via32(double *As, double *Bs, double *Xs);

// bounded spins of the in-launch hand-offs (then status[1]: re-solve without them)
#ifndef BA_BACK_SPIN_MAX
#define BA_BACK_SPIN_MAX 400000u
#endif
// kflag (one-launch hand-off, may be null): workgroup 0 publishes L_kk^-1 and
// y_k (write-through stores, then flag k = epoch) and the panel workgroups
// take them from there instead of updating and factoring A_kk themselves --
// the same bits (workgroup 0's factor is the one they would recompute), with
// the panel's own pending update overlapping workgroup 0's factor.  A panel
// workgroup only waits on workgroup 0 of its column, which has a lower index
// (dispatched first); a spin that gives up sets status[1] and the host
// re-solves with kflag = null.
__device__ __forceinline__ void factor_step_body(double *__restrict__ S, long long lds, int k,
                                                 const int *__restrict__ pan, int T,
                                                 const int *__restrict__ prev, int Tp,
                                                 double *__restrict__ linv,
                                                 double *__restrict__ rhs,
                                                 double *__restrict__ y,
                                                 double *__restrict__ status, int b, int sep0,
                                                 unsigned *__restrict__ kflag, unsigned epoch)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP, *Cs = sm + 2 * NB * LP;
    __shared__ double yk[NB], rk[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x;
    const bool kin = Tp > 0 && prev[0] == k;   // column k-1 reaches row k
    d4 acc[2][2];
    FS_ST(0);
    if (b > T) {
        // trailing pairs of column k-1 below row k (k_syrk's enumeration over
        // prev without k)
        const int *pl = prev + (kin ? 1 : 0);
        const int Tr = Tp - (kin ? 1 : 0);
        int q = b - T - 1, jj = 0;
        while (q >= Tr - jj) {
            q -= Tr - jj;
            jj++;
        }
        const int j = pl[jj], i = pl[jj + q];
        double va[16], vb[16], vc[16];
        fetch_tile(S, lds, i, k - 1, va);
        fetch_tile(S, lds, j, k - 1, vb);
        fetch_tile(S, lds, i, j, vc);
        put_tile(As, va, false);
        put_tile(Bs, vb, false);
        put_tile(Cs, vc, false);
        __syncthreads();
        mfma_64x64(As, Bs, acc);
        acc_to_lds(acc, Cs, -1.0, true);
        __syncthreads();
        store_tile(S, lds, i, j, Cs);
        FS_END();
        return;
    }
    const int i = b > 0 ? pan[b - 1] : k;
    const bool hand = kflag != nullptr && b > 0;   // a panel taking L_kk^-1 / y_k from workgroup 0
    // every tile this workgroup reads, fetched at once (one memory latency
    // instead of three dependent ones): A_ik, L_k,k-1, A_kk, L_i,k-1
    double vc[16], va[16], vb[16], vk[16];
    if (b > 0) fetch_tile(S, lds, i, k, vc);
    if (kin) fetch_tile(S, lds, k, k - 1, vb);
    if (!hand) fetch_tile(S, lds, k, k, vk);
    bool iin = false;   // column k-1 reaches row i (panel tiles only): a wave-wide search
    if (b > 0 && kin) {
        const int lane = tid & 63;
        for (int t0 = 1; t0 < Tp && !iin; t0 += 64)
            iin = __any(t0 + lane < Tp && prev[t0 + lane] == i);
    }
    if (iin) fetch_tile(S, lds, i, k - 1, va);
    if (!hand && tid < NB) rk[tid] = rhs[(long long)NB * k + tid];
    if (b > 0) put_tile(Cs, vc, false);
    if (iin) put_tile(As, va, false);
    if (kin) put_tile(Bs, vb, false);
    __syncthreads();
    if (iin) {   // A_ik's pending update of column k-1
        mfma_64x64(As, Bs, acc);
        __syncthreads();
        acc_to_lds(acc, Cs, -1.0, true);
    }
    if (hand) {
        if (tid < 64) {   // wave 0 waits for workgroup 0's flag
            for (unsigned spins = 0;; spins++) {
                const unsigned f = __hip_atomic_load((const gu32_t *)(kflag + k), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if (f == epoch) break;
                if (spins >= BA_BACK_SPIN_MAX) {
                    if (tid == 0) status[1] = 1.0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        {   // L_kk^-1 (row-major, write-through) -> Bs, y_k -> yk (agent-scope loads)
            const double *lo = linv + (long long)NB * NB * k;
            const int c = tid & 63, r0 = tid >> 6;
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; u++) v[u] = ldg<true>(lo + (r0 + 4 * u) * NB + c);
#pragma unroll
            for (int u = 0; u < 16; u++) Bs[(r0 + 4 * u) * LP + c] = v[u];
            if (tid < NB) yk[tid] = ldg<true>(y + (long long)NB * k + tid);
        }
        __syncthreads();
        FS_ST(1);
        FS_ST(2);
    } else {
    // A_kk and its pending update
    if (kin) mfma_64x64(Bs, Bs, acc);
    __syncthreads();
    put_tile(As, vk, false);
    __syncthreads();
    if (kin) {
        acc_to_lds(acc, As, -1.0, true);
        __syncthreads();
    }
    FS_ST(1);
    const bool ok = potrf64_via32(As, Bs, As + 32);   // scratch: A's upper-right block
    FS_ST(2);
    gemv64(Bs, rk, part, yk, 1.0);            // y_k = L^-1 r_k
    if (b == 0 && kflag) {   // published for the column's panel workgroups
        double *lo = linv + (long long)NB * NB * k;
        for (int q = tid; q < NB * NB; q += blockDim.x)
            stg<true>(lo + q, Bs[(q >> 6) * LP + (q & 63)]);
        if (tid < NB) stg<true>(y + (long long)NB * k + tid, yk[tid]);
        if (tid == 0 && !ok) status[0] = 1.0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store((gu32_t *)(kflag + k), epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        FS_ST(3);
        FS_END();
        return;
    }
    if (b == 0) {
        // L_kk is NOT stored back to S(k, k): the panel workgroups of this
        // launch read A_kk from there, and one that starts after this store
        // (a busy GPU: not every workgroup is resident at once) would factor
        // L_kk instead of A_kk.  Nothing reads L_kk later (the backward solve
        // takes L_kk^-1 from linv, the next columns only off-diagonal tiles).
        double *lo = linv + (long long)NB * NB * k;
        for (int q = tid; q < NB * NB; q += blockDim.x) lo[q] = Bs[(q >> 6) * LP + (q & 63)];
        if (tid < NB) y[(long long)NB * k + tid] = yk[tid];
        if (tid == 0 && !ok) status[0] = 1.0;
        FS_ST(3);
        FS_END();
        return;
    }
    }   // (!hand)
    mfma_64x64(Cs, Bs, acc);   // L_ik[r][c] = sum_t A_ik[r][t] Li[c][t]
    __syncthreads();
    acc_to_lds(acc, Cs, 1.0, false);
    __syncthreads();
    store_tile(S, lds, i, k, Cs);
    double ri[1];
    gemv64(Cs, yk, part, nullptr, 1.0, ri);   // (L_ik y_k)[tid] for tid < 64
    if (tid < NB && i < sep0) rhs[(long long)NB * i + tid] -= ri[0];
    FS_ST(3);
    FS_END();
}

// Runner mode (k_env_runner beside the column launches; the default,
// VLGBA_ENV_RUNNER=0 turns it off): a
// persistent workgroup per run of columns [k0, kend) factors every diagonal
// tile and forms the first panel tile L_k+1,k itself, so the column launches
// lose workgroup 0 and that panel.  The tiles the two exchange inside a launch
// go through sc1 stores / loads and a flag each (epoch = fac_epoch):
//   lflag[k]   L_k,k-1 stored by the runner (the panels' pending update reads it)
//   dflag[k]   A_kk's last trailing update (column k-2) stored
//   uflag[k+1] A_k+1,k's pending update of column k-1 stored (the runner's panel)
//   pflag[k+1] r_k+1's update by column k-1's panel stored (before the runner's)
// (a profile: column c reaches row i for every c from row i's first column on,
// so these are the only writes the runner waits for; every other write it
// reads was made by a launch that ended before one of those flags was set).
struct env_rm {
    unsigned *lflag, *dflag, *uflag, *pflag;
    unsigned *rto;   // a runner hand-off gave up (the host turns this context's runner off)
    int kend;   // the run's end column (exclusive); 0: not in runner mode
};

// wave 0 spins on flag[idx] == epoch (bounded; timeout: status[1] and the
// runner's own word *rto); all waves then pass a barrier.  Returns false on a
// timeout.
__device__ __forceinline__ bool env_wait(const unsigned *flag, int idx, unsigned epoch,
                                         double *status, unsigned *rto)
{
    __shared__ int to;
    const int tid = threadIdx.x;
    if (tid < 64) {
        bool ok = false;
        for (unsigned spins = 0; spins < BA_BACK_SPIN_MAX; spins++) {
            const unsigned f = __hip_atomic_load((const gu32_t *)(flag + idx), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            if (f == epoch) {
                ok = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (tid == 0) {
            to = ok ? 0 : 1;
            if (!ok) {
                status[1] = 1.0;
                __hip_atomic_store((gu32_t *)rto, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    return to == 0;
}

__device__ __forceinline__ void env_publish(unsigned *flag, int idx, unsigned epoch)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store((gu32_t *)(flag + idx), epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// factor_step_body with the in-launch hand-off on two LDS tiles instead of
// three (two workgroups per CU): the pending updates' operands come straight
// from S (mfma_64x64_glb), workgroup 0 factors in As -> Bs, a panel keeps
// A_ik in As and L_kk^-1 in Bs, a trailing pair its C tile in As.  The same
// operations in the same order: bit-identical to factor_step_body.
__device__ __forceinline__ void factor_step_two(double *__restrict__ S, long long lds, int k,
                                                const int *__restrict__ pan, int T,
                                                const int *__restrict__ prev, int Tp,
                                                double *__restrict__ linv,
                                                double *__restrict__ rhs,
                                                double *__restrict__ y,
                                                double *__restrict__ status, int b, int sep0,
                                                unsigned *__restrict__ kflag, unsigned epoch,
                                                int ntr, int tstride, env_rm R = env_rm{})
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    __shared__ double yk[NB], rk[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x;
    const bool kin = Tp > 0 && prev[0] == k;   // column k-1 reaches row k
    d4 acc[2][2];
    FS_ST(0);
    if (b > T) {
        // trailing pairs q = b - T - 1 + u tstride (< ntr) of column k-1
        // below row k, one after another: fewer workgroups than pairs keeps
        // them off most CUs, so the diagonal factor's chain seldom shares one
        const int *pl = prev + (kin ? 1 : 0);
        const int Tr = Tp - (kin ? 1 : 0);
        for (int q0 = b - T - 1; q0 < ntr; q0 += tstride) {
            int q = q0, jj = 0;
            while (q >= Tr - jj) {
                q -= Tr - jj;
                jj++;
            }
            const int j = pl[jj], i = pl[jj + q];
            double vc[16];
            fetch_tile(S, lds, i, j, vc);
            mfma_64x64_glb(S, lds, i, j, k - 1, acc);
            put_tile(As, vc, false);
            __syncthreads();
            acc_to_lds(acc, As, -1.0, true);
            __syncthreads();
            if (R.kend && i == k + 1 && j == k + 1 && k + 1 < R.kend) {
                // A_k+1,k+1's last trailing update: the runner reads it at column k+1
                store_tile_sc(S, lds, i, j, As);
                env_publish(R.dflag, k + 1, epoch);
            } else {
                store_tile(S, lds, i, j, As);
            }
            __syncthreads();   // As read by every thread before the next pair's put
        }
        FS_END();
        return;
    }
    if (b == 0 && R.kend) {   // the runner factors A_kk
        FS_END();
        return;
    }
    if (b == 0) {   // A_kk's pending update, factor, L_kk^-1, y_k; published
        double vk[16];
        fetch_tile(S, lds, k, k, vk);
        if (tid < NB) rk[tid] = rhs[(long long)NB * k + tid];
        if (kin) mfma_64x64_glb(S, lds, k, k, k - 1, acc);
        put_tile(As, vk, false);
        __syncthreads();
        if (kin) {
            acc_to_lds(acc, As, -1.0, true);
            __syncthreads();
        }
        FS_ST(1);
        const bool ok = potrf64_via32(As, Bs, As + 32);
        FS_ST(2);
        gemv64(Bs, rk, part, yk, 1.0);   // y_k = L^-1 r_k
        double *lo = linv + (long long)NB * NB * k;
        for (int q = tid; q < NB * NB; q += blockDim.x)
            stg<true>(lo + q, Bs[(q >> 6) * LP + (q & 63)]);
        if (tid < NB) stg<true>(y + (long long)NB * k + tid, yk[tid]);
        if (tid == 0 && !ok) status[0] = 1.0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store((gu32_t *)(kflag + k), epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        FS_ST(3);
        FS_END();
        return;
    }
    // a panel tile: A_ik and its pending update, then L_ik = A_ik L_kk^-T
    const int i = pan[b - 1];
    double vc[16];
    fetch_tile(S, lds, i, k, vc);
    bool iin = false;   // column k-1 reaches row i: a wave-wide search
    if (kin) {
        const int lane = tid & 63;
        for (int t0 = 1; t0 < Tp && !iin; t0 += 64)
            iin = __any(t0 + lane < Tp && prev[t0 + lane] == i);
    }
    const bool lrun = R.kend && i == k + 1 && k + 1 < R.kend;   // the runner's panel
    if (lrun && !iin) {   // no pending update: the runner reads A_k+1,k as it is
        FS_END();
        return;
    }
    if (iin && R.kend) {   // L_k,k-1 is the runner's
        if (!env_wait(R.lflag, k, epoch, status, R.rto)) return;
        mfma_64x64_glb<true>(S, lds, i, k, k - 1, acc);
    } else if (iin) {
        mfma_64x64_glb(S, lds, i, k, k - 1, acc);
    }
    put_tile(As, vc, false);
    __syncthreads();
    if (iin) acc_to_lds(acc, As, -1.0, true);
    if (lrun) {   // A_k+1,k after its pending update, for the runner
        __syncthreads();
        store_tile_sc(S, lds, i, k, As);
        env_publish(R.uflag, k + 1, epoch);
        FS_END();
        return;
    }
    if (tid < 64) {   // wave 0 waits for workgroup 0's flag
        for (unsigned spins = 0;; spins++) {
            const unsigned f = __hip_atomic_load((const gu32_t *)(kflag + k), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            if (f == epoch) break;
            if (spins >= BA_BACK_SPIN_MAX) {
                if (tid == 0) status[1] = 1.0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    {   // L_kk^-1 (row-major, write-through) -> Bs, y_k -> yk (agent-scope loads)
        const double *lo = linv + (long long)NB * NB * k;
        const int c = tid & 63, r0 = tid >> 6;
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = ldg<true>(lo + (r0 + 4 * u) * NB + c);
#pragma unroll
        for (int u = 0; u < 16; u++) Bs[(r0 + 4 * u) * LP + c] = v[u];
        if (tid < NB) yk[tid] = ldg<true>(y + (long long)NB * k + tid);
    }
    __syncthreads();
    FS_ST(1);
    FS_ST(2);
    mfma_64x64(As, Bs, acc);   // L_ik[r][c] = sum_t A_ik[r][t] Li[c][t]
    __syncthreads();
    acc_to_lds(acc, As, 1.0, false);
    __syncthreads();
    store_tile(S, lds, i, k, As);
    double ri[1];
    gemv64(As, yk, part, nullptr, 1.0, ri);   // (L_ik y_k)[tid] for tid < 64
    if (R.kend && i == k + 2 && k + 2 < R.kend) {   // the runner updates r_k+2 next
        if (tid < NB) {
            double *rp = rhs + (long long)NB * i + tid;
            stg<true>(rp, ldg<true>(rp) - ri[0]);
        }
        env_publish(R.pflag, k + 2, epoch);
    } else if (tid < NB && i < sep0) {
        rhs[(long long)NB * i + tid] -= ri[0];
    }
    FS_ST(3);
    FS_END();
}

__global__ __launch_bounds__(256) void k_factor_step(double *__restrict__ S, long long lds, int k,
                                                     const int *__restrict__ pan, int T,
                                                     const int *__restrict__ prev, int Tp,
                                                     double *__restrict__ linv,
                                                     double *__restrict__ rhs,
                                                     double *__restrict__ y,
                                                     double *__restrict__ status,
                                                     unsigned *__restrict__ kflag, unsigned epoch,
                                                     int ntr, int tstride, env_rm R)
{
    if (kflag)
        factor_step_two(S, lds, k, pan, T, prev, Tp, linv, rhs, y, status, blockIdx.x, INT_MAX,
                        kflag, epoch, ntr, tstride, R);
    else
        factor_step_body(S, lds, k, pan, T, prev, Tp, linv, rhs, y, status, blockIdx.x, INT_MAX,
                         nullptr, 0);
}

// one step of every arc of the nested dissection: column k[t] of arc t takes
// workgroups [b0[t], b0[t+1]) (k_factor_step's roles), pan / prev as offsets
// into the panel list
// Workgroup order (grouped, the default): every arc's workgroup 0 first, then
// every arc's panel tiles, then every arc's trailing pairs (pb / tb: prefix
// counts of the panels / trailing pairs over the arcs).  Arc-major order
// (b0, VLGBA_ND_GROUPED=0) puts arc 1's workgroup 0 behind all of arc 0's
// trailing pairs: once those outnumber the free workgroup slots, arc 1's
// diagonal factor -- the chain of its step -- starts only when the first of
// them retire.  The roles are the same either way (bit-identical).
struct nd_step {
    int np, grouped;
    int k[BA_ND_MAX], T[BA_ND_MAX], Tp[BA_ND_MAX], pofs[BA_ND_MAX], qofs[BA_ND_MAX];
    int ntr[BA_ND_MAX], ts[BA_ND_MAX];   // trailing pairs / their workgroups (stride)
    int kend[BA_ND_MAX];                 // runner mode: arc t's end column (else 0)
    int b0[BA_ND_MAX + 1], pb[BA_ND_MAX + 1], tb[BA_ND_MAX + 1];
};

__global__ __launch_bounds__(256) void k_factor_multi(double *__restrict__ S, long long lds,
                                                      const int *__restrict__ pan_list,
                                                      nd_step P, int sep0,
                                                      double *__restrict__ linv,
                                                      double *__restrict__ rhs,
                                                      double *__restrict__ y,
                                                      double *__restrict__ status,
                                                      unsigned *__restrict__ kflag,
                                                      unsigned epoch, env_rm R)
{
    const int b = blockIdx.x, np = P.np;
    int t = 0, role;
    if (!P.grouped) {
        while (t + 1 < np && b >= P.b0[t + 1]) t++;
        role = b - P.b0[t];
    } else if (b < np) {   // workgroup 0 of arc b
        t = b;
        role = 0;
    } else if (b < np + P.pb[np]) {   // a panel tile
        const int q = b - np;
        while (t + 1 < np && q >= P.pb[t + 1]) t++;
        role = 1 + q - P.pb[t];
    } else {   // a trailing pair
        const int q = b - np - P.pb[np];
        while (t + 1 < np && q >= P.tb[t + 1]) t++;
        role = 1 + P.T[t] + q - P.tb[t];
    }
    R.kend = P.kend[t];
    if (kflag)
        factor_step_two(S, lds, P.k[t], pan_list + P.pofs[t], P.T[t], pan_list + P.qofs[t],
                        P.Tp[t], linv, rhs, y, status, role, sep0, kflag, epoch, P.ntr[t],
                        P.ts[t], R);
    else
        factor_step_body(S, lds, P.k[t], pan_list + P.pofs[t], P.T[t], pan_list + P.qofs[t],
                         P.Tp[t], linv, rhs, y, status, role, sep0, nullptr, 0);
}

// ---------------------------------------------------------------------------
// k_env_runner: one persistent workgroup per run of columns [k0[t], k1[t])
// (the nested dissection's arcs side by side, or the natural order's one run),
// launched on the side stream beside the per-column launches.  Per column k:
//   A_kk (after its last trailing update: dflag[k] when column k-2 reaches row
//   k) and column k-1's pending update from the workgroup's own LDS copy of
//   L_k,k-1; the factor, L_kk^-1, y_k, published (kflag[k]) exactly as
//   factor_step_two's workgroup 0; then, when row k+1 is in column k's panel,
//   L_k+1,k = A_k+1,k L_kk^-T (after column k-1's panel's r_k+1 update, pflag,
//   and its pending update, uflag) stored with sc1, r_k+1 -= L_k+1,k y_k, lflag[k+1] --
//   the tile stays in LDS for column k+1.  Every tile sees the same operations
//   in the same order as in the column launches alone: bit-identical.  A wait
//   that gives up sets status[1] and ends the workgroup (the host re-solves
//   without hand-offs).
// ---------------------------------------------------------------------------
struct env_runs {
    int np;
    int k0[BA_ND_MAX], k1[BA_ND_MAX];
};

__global__ __launch_bounds__(256) void k_env_runner(double *S, long long lds,
                                                    const int *__restrict__ pan_ptr,
                                                    const int *__restrict__ pan_list, env_runs Rn,
                                                    double *linv, double *rhs, double *y,
                                                    double *status, unsigned *kflag,
                                                    env_rm R, unsigned epoch)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    double *Ls = sm + 2 * NB * LP, *Ps = sm + 3 * NB * LP;
    __shared__ double yk[NB], rk[NB];
    __shared__ double part[4][NB];
    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    if (t >= Rn.np) return;
    const int k0 = Rn.k0[t], k1 = Rn.k1[t];
    bool have_l = false;   // Ls holds L_k,k-1
    d4 acc[2][2];
    // row i among column c's panel rows (a wave-wide search, every wave)
    auto reaches = [&](int c, int i) {
        const int q0 = pan_ptr[c], n = pan_ptr[c + 1] - q0;
        bool f = false;
        for (int u = 0; u < n && !f; u += 64) f = __any(u + lane < n && pan_list[q0 + u + lane] == i);
        return f;
    };
    for (int k = k0; k < k1; k++) {
        const int p0 = pan_ptr[k], T = pan_ptr[k + 1] - p0;
        if (k - 2 >= k0 && reaches(k - 2, k) && !env_wait(R.dflag, k, epoch, status, R.rto)) return;
        double vk[16];
        fetch_tile_sc(S, lds, k, k, vk);
        if (tid < NB) rk[tid] = ldg<true>(rhs + (long long)NB * k + tid);
        if (have_l) mfma_64x64(Ls, Ls, acc);
        __syncthreads();
        put_tile(As, vk, false);
        __syncthreads();
        if (have_l) {
            acc_to_lds(acc, As, -1.0, true);
            __syncthreads();
        }
        const bool ok = potrf64_via32(As, Bs, As + 32);
        gemv64(Bs, rk, part, yk, 1.0);   // y_k = L^-1 r_k
        {
            double *lo = linv + (long long)NB * NB * k;
            for (int q = tid; q < NB * NB; q += blockDim.x)
                stg<true>(lo + q, Bs[(q >> 6) * LP + (q & 63)]);
            if (tid < NB) stg<true>(y + (long long)NB * k + tid, yk[tid]);
            if (tid == 0 && !ok) status[0] = 1.0;
        }
        env_publish(kflag, k, epoch);
        have_l = false;
        if (k + 1 < k1 && T > 0 && pan_list[p0] == k + 1) {
            // launch k-1 ended (its trailing update of A_k+1,k and its panel's
            // r_k+1 update), and column k-1's pending update of A_k+1,k stored
            if (k > k0 && reaches(k - 1, k + 1)) {
                // column k-1's panel updated r_k+1; its pending update of A_k+1,k
                if (!env_wait(R.pflag, k + 1, epoch, status, R.rto)) return;
                const bool kin = pan_ptr[k] > pan_ptr[k - 1] && pan_list[pan_ptr[k - 1]] == k;
                if (kin && !env_wait(R.uflag, k + 1, epoch, status, R.rto)) return;
            }
            double va[16];
            fetch_tile_sc(S, lds, k + 1, k, va);
            put_tile(Ps, va, false);
            __syncthreads();
            mfma_64x64(Ps, Bs, acc);   // L[r][c] = sum_t A[r][t] Li[c][t]
            __syncthreads();
            acc_to_lds(acc, Ps, 1.0, false);
            __syncthreads();
            store_tile_sc(S, lds, k + 1, k, Ps);
            double ri[1];
            gemv64(Ps, yk, part, nullptr, 1.0, ri);   // (L y_k)[tid] for tid < 64
            if (tid < NB) {
                double *rp = rhs + (long long)NB * (k + 1) + tid;
                stg<true>(rp, ldg<true>(rp) - ri[0]);
            }
            env_publish(R.lflag, k + 1, epoch);
            double *sw = Ls;
            Ls = Ps;
            Ps = sw;
            have_l = true;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// The arcs' contribution to the separator block (nested dissection): record
// (pair (i, j), arc columns klist[kofs .. kofs+kcnt)) forms
//     P = sum_k L_ik L_jk^T        (and for i == j:  g = sum_k L_ik y_k)
// over its columns in ascending order (one MFMA accumulator chain), stored
// column-major in part[rec][64*64] (+ 64).  Chunks of the arc columns keep
// every record short enough to fill the chip in one wave.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sep_update(const double *__restrict__ S, long long lds,
                                                    const int *__restrict__ pair,
                                                    const int *__restrict__ rec,
                                                    const int *__restrict__ klist,
                                                    const double *__restrict__ y,
                                                    double *__restrict__ part)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    __shared__ double ys[NB];
    const int tid = threadIdx.x, r = tid & 63, cq = tid >> 6;
    const int pr = rec[3 * blockIdx.x], kofs = rec[3 * blockIdx.x + 1], kcnt = rec[3 * blockIdx.x + 2];
    const int i = pair[2 * pr], j = pair[2 * pr + 1];
    d4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int z = 0; z < 2; z++) acc[x][z] = d4{0.0, 0.0, 0.0, 0.0};
    double g = 0.0;   // thread (r, cq): sum over its quarter of the columns
    for (int q = 0; q < kcnt; q++) {
        const int k = klist[kofs + q];
        __syncthreads();   // previous tiles consumed
        load_tile(S, lds, i, k, As);
        if (i != j) load_tile(S, lds, j, k, Bs);
        if (i == j && tid < NB) ys[tid] = y[(long long)NB * k + tid];
        __syncthreads();
        mfma_64x64_acc(As, i == j ? As : Bs, acc);
        if (i == j) {
            double s = 0.0;
#pragma unroll
            for (int c = 16 * cq; c < 16 * cq + 16; c++) s += As[r * LP + c] * ys[c];
            g += s;
        }
    }
    __syncthreads();
    acc_to_lds(acc, As, 1.0, false);
    __syncthreads();
    double *out = part + (size_t)blockIdx.x * (NB * NB + NB);
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int c = cq + 4 * u;
        out[c * NB + r] = As[r * LP + c];
    }
    if (i == j) {
        __shared__ double gp[4][NB];
        gp[cq][r] = g;
        __syncthreads();
        if (tid < NB) out[NB * NB + tid] = ((gp[0][tid] + gp[1][tid]) + gp[2][tid]) + gp[3][tid];
    }
}

// A_ij -= sum of the pair's records (in record order); rhs_i -= sum of g
__global__ __launch_bounds__(256) void k_sep_reduce(double *__restrict__ S, long long lds,
                                                    const int *__restrict__ pair,
                                                    const int *__restrict__ pptr,
                                                    const double *__restrict__ part,
                                                    double *__restrict__ rhs)
{
    const int p = blockIdx.x, tid = threadIdx.x, r = tid & 63, cq = tid >> 6;
    const int i = pair[2 * p], j = pair[2 * p + 1];
    const int e0 = pptr[p], e1 = pptr[p + 1];
    double s[16];
#pragma unroll
    for (int u = 0; u < 16; u++) s[u] = 0.0;
    double g = 0.0;
    for (int e = e0; e < e1; e++) {
        const double *src = part + (size_t)e * (NB * NB + NB);
#pragma unroll
        for (int u = 0; u < 16; u++) s[u] += src[(cq + 4 * u) * NB + r];
        if (i == j && tid < NB) g += src[NB * NB + tid];
    }
    double *base = S + (long long)NB * i + lds * (long long)NB * j;
#pragma unroll
    for (int u = 0; u < 16; u++) base[r + lds * (cq + 4 * u)] -= s[u];
    if (i == j && tid < NB) rhs[(long long)NB * i + tid] -= g;
}

// da (camera order, ld..lds zero) from the row-ordered solution
__global__ void k_nd_scatter(const int *__restrict__ prow, const double *__restrict__ x,
                             double *__restrict__ da, long long lds)
{
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= lds) return;
    const int r = prow[c];
    da[c] = r >= 0 ? x[r] : 0.0;
}

// ---------------------------------------------------------------------------
// backward solve step k: x_k = L_kk^-T z_k; z_j -= L_kj^T x_k, j in [j0, k)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_backward(const double *__restrict__ S, long long lds,
                                                  int k, int j0,
                                                  const double *__restrict__ linv,
                                                  double *__restrict__ z, double *__restrict__ x)
{
    __shared__ double xs[NB], zk[NB];
    __shared__ double part[4][NB];
    __shared__ double Lt[NB * LP];
    const int j = j0 + blockIdx.x, tid = threadIdx.x;
    const double *lo = linv + (long long)NB * NB * k;  // row-major L^-1
    load_rowmajor(lo, Lt);
    if (tid < NB) zk[tid] = z[(long long)NB * k + tid];
    __syncthreads();
    {   // x_k[c] = sum_{r >= c} Li[r][c] z_k[r]: thread (c, quarter)
        const int c = tid & 63, qr = tid >> 6;
        double s = 0.0;
        for (int r = 16 * qr; r < 16 * qr + 16; r++)
            if (r >= c) s += Lt[r * LP + c] * zk[r];
        part[qr][c] = s;
    }
    __syncthreads();
    if (tid < NB) xs[tid] = ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
    __syncthreads();
    if (j == k) {
        if (tid < NB) x[(long long)NB * k + tid] = xs[tid];
        return;
    }
    // z_j[c] -= sum_r L_kj[r][c] x_k[r]: stage L_kj (coalesced), thread (c, quarter)
    load_tile(S, lds, k, j, Lt);
    __syncthreads();
    const int c = tid & 63, qr = tid >> 6;
    double s = 0.0;
#pragma unroll
    for (int r = 16 * qr; r < 16 * qr + 16; r++) s += Lt[r * LP + c] * xs[r];
    part[qr][c] = s;
    __syncthreads();
    if (tid < NB)
        z[(long long)NB * j + tid] -= ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
}

// ---------------------------------------------------------------------------
// The envelope's backward solve in ONE launch (the per-column k_backward
// launches sat at the launch floor).  Workgroup w takes tile column
// j = nt-1-w (top first): z_j = y_j - sum over the envelope rows k > j (k
// descending, the order of the per-column launches: bit-identical) of
// L_kj^T x_k, then x_j = L_jj^-T z_j, published as 128 epoch-tagged 8-byte
// write-through granules (cdna_hip_programming.md Guideline 16, R2); each x_k
// is swept by wave 0 until every tag matches.  Used when every column is
// co-resident (one workgroup per CU by LDS: nt <= CUs); a spin that never
// ends sets the timeout word status[1] instead of hanging.  Each tile (k, j) is loaded while
// the wave waits for x_k.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_backward_all(const double *__restrict__ S, long long lds,
                                                      int nt, const int *__restrict__ pan_ptr,
                                                      const int *__restrict__ pan,
                                                      const double *__restrict__ linv,
                                                      const double *__restrict__ z,
                                                      double *__restrict__ x,
                                                      unsigned long long *__restrict__ xg,
                                                      unsigned epoch, double *status)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *Lt = sm, *Li = sm + NB * LP;
    __shared__ __attribute__((aligned(16))) double zj[NB], xs[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int j = nt - 1 - (int)blockIdx.x;
    load_rowmajor(linv + (long long)NB * NB * j, Li);
    if (tid < NB) zj[tid] = z[(long long)NB * j + tid];
    const int c = tid & 63, qr = tid >> 6;
    for (int idx = pan_ptr[j + 1] - 1; idx >= pan_ptr[j]; idx--) {
        const int k = pan[idx];
        __syncthreads();   // Lt / xs of the previous k consumed
        load_tile(S, lds, k, j, Lt);
        if (wv == 0) {
            const unsigned long long *g = xg + 128 * (size_t)k;
            unsigned long long v0 = 0, v1 = 0;
            for (unsigned spins = 0;; spins++) {
                v0 = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v1 = __hip_atomic_load(g + 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__all((unsigned)(v0 >> 32) == epoch && (unsigned)(v1 >> 32) == epoch)) break;
                if (spins >= BA_BACK_SPIN_MAX) {
                    if (lane == 0) status[1] = 1.0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            unsigned *xu = reinterpret_cast<unsigned *>(xs);
            xu[lane] = (unsigned)v0;
            xu[64 + lane] = (unsigned)v1;
        }
        __syncthreads();
        // z_j[c] -= sum_r L_kj[r][c] x_k[r]: thread (c, quarter), as k_backward
        double s = 0.0;
#pragma unroll
        for (int r = 16 * qr; r < 16 * qr + 16; r++) s += Lt[r * LP + c] * xs[r];
        part[qr][c] = s;
        __syncthreads();
        if (tid < NB) zj[tid] -= ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
    }
    __syncthreads();
    {   // x_j[c] = sum_{r >= c} Li[r][c] z_j[r]: thread (c, quarter), as k_backward
        double s = 0.0;
        for (int r = 16 * qr; r < 16 * qr + 16; r++)
            if (r >= c) s += Li[r * LP + c] * zj[r];
        part[qr][c] = s;
    }
    __syncthreads();
    if (tid < NB) {
        const double xv = ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
        xs[tid] = xv;
        x[(long long)NB * j + tid] = xv;
    }
    __syncthreads();
    if (wv == 0) {
        const unsigned *xu = reinterpret_cast<const unsigned *>(xs);
        unsigned long long *g = xg + 128 * (size_t)j;
        __hip_atomic_store(g + lane, ((unsigned long long)epoch << 32) | xu[lane],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 64 + lane, ((unsigned long long)epoch << 32) | xu[64 + lane],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// Block cyclic reduction for a tile-tridiagonal S (co-visibility band narrower
// than one tile: tile row i couples only with tiles i-1, i+1).  This is the
// Cholesky factorisation of S in odd-even (nested-dissection) order: at each
// level the even positions e of the active tile list are eliminated in
// parallel; their neighbours p < e < q are kept and coupled through e.  Per
// eliminated tile e (L_e = chol(D_e)):
//     Lp_e = L(p, e) = C(p, e) L_e^-T,   Lq_e = L(q, e) = C(q, e) L_e^-T,
//     y_e  = L_e^-1 r_e
// per kept tile k with eliminated neighbours e- < k < e+ and next kept k2:
//     D_k -= Lq_{e-} Lq_{e-}^T + Lp_{e+} Lp_{e+}^T,
//     r_k -= Lq_{e-} y_{e-} + Lp_{e+} y_{e+},
//     C(k2, k) = -Lq_{e+} Lp_{e+}^T          (fill between the kept tiles)
// log2(nt) levels instead of nt sequential tile steps.  Back substitution in
// reverse level order: x_e = L_e^-T (y_e - Lp_e^T x_p - Lq_e^T x_q).
// C(i, j), i > j, lives in S tile (i, j); Lp / Lq in crL[2][nt][64*64].
// ---------------------------------------------------------------------------
// Rows 32h .. 32h+31 of the 64x64 product acc = As[r][:] . Bs[c][:] (K = 64):
// wave w owns rows 32h + 16(w>>1) .. +15, cols 32(w&1) .. +31 (two 16x16
// MFMA tiles), half the MFMA chain of mfma_64x64.
__device__ __forceinline__ void mfma_half(const double *As, const double *Bs, int h, d4 acc[2],
                                          bool zero)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * h + 16 * (w >> 1), c0 = 32 * (w & 1);
    const int li = lane & 15, lk = lane >> 4;
    if (zero) acc[0] = acc[1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int s = 0; s < NB / 4; s++) {
        const int kk = 4 * s + lk;
        const double a0 = As[(r0 + li) * LP + kk];
        const double b0 = Bs[(c0 + li) * LP + kk];
        const double b1 = Bs[(c0 + 16 + li) * LP + kk];
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
    }
}

// mfma_half's result: T[r][c] = scale * acc (+ T[r][c] if add)
__device__ __forceinline__ void half_to_lds(const d4 acc[2], double *T, int h, double scale,
                                            bool add)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * h + 16 * (w >> 1), c0 = 32 * (w & 1);
#pragma unroll
    for (int y = 0; y < 2; y++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = r0 + (lane >> 4) + 4 * q, c = c0 + 16 * y + (lane & 15);
            const double v = scale * acc[y][q];
            T[r * LP + c] = add ? T[r * LP + c] + v : v;
        }
}

// rows 32h .. +31 of LDS T[r][c] -> row-major dst[r*64 + c]
__device__ __forceinline__ void store_rowmajor_half(double *__restrict__ dst, const double *T,
                                                    int h)
{
    const int c = threadIdx.x & 63, r0 = 32 * h + (threadIdx.x >> 6);
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = T[(r0 + 4 * u) * LP + c];
#pragma unroll
    for (int u = 0; u < 8; u++) dst[(r0 + 4 * u) * NB + c] = v[u];
}

// rows 32h .. +31 of S tile (ti, tj) <-> LDS T[r][c]; thread (row, 8 columns)
__device__ __forceinline__ void load_tile_half(const double *__restrict__ S, long long lds, int ti,
                                               int tj, double *T, int h)
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = 32 * h + (threadIdx.x & 31), c0 = threadIdx.x >> 5;
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = base[r + lds * (c0 + 8 * u)];
#pragma unroll
    for (int u = 0; u < 8; u++) T[r * LP + c0 + 8 * u] = v[u];
}

__device__ __forceinline__ void store_tile_half(double *__restrict__ S, long long lds, int ti,
                                                int tj, const double *T, int h)
{
    double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    const int r = 32 * h + (threadIdx.x & 31), c0 = threadIdx.x >> 5;
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = T[r * LP + c0 + 8 * u];
#pragma unroll
    for (int u = 0; u < 8; u++) base[r + lds * (c0 + 8 * u)] = v[u];
}

// Factor step of a level.  split = 0: one workgroup per eliminated tile does
// everything.  split = 1 (levels narrow enough that 5 workgroups per tile fit
// the chip): workgroup role 0 factors D_e and writes L_e^-1 and y_e; roles
// 1-2 (rows halves of Lp_e) and 3-4 (of Lq_e) redo the same factorisation --
// deterministic, bit-identical -- with their C tile loaded alongside, and form
// their 32 rows of the panel.  The critical path loses both 64x64 panel GEMMs.
__global__ __launch_bounds__(256) void k_cr_factor(double *__restrict__ S, long long lds,
                                                   const int *__restrict__ elim, int nt,
                                                   double *__restrict__ linv,
                                                   double *__restrict__ crL,
                                                   const double *__restrict__ rhs,
                                                   double *__restrict__ y,
                                                   double *__restrict__ status, int split)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP, *Cs = sm + 2 * NB * LP;
    __shared__ double rk[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x;
    const int x = split ? blockIdx.x / 5 : blockIdx.x, role = split ? blockIdx.x % 5 : -1;
    const int e = elim[3 * x], p = elim[3 * x + 1], q = elim[3 * x + 2];
    if ((role == 1 || role == 2) && p < 0) return;
    if ((role == 3 || role == 4) && q < 0) return;
    {
        double va[16], vc[16];
        fetch_tile(S, lds, e, e, va);
        if (role > 0) {   // C(p, e) = tile(e, p)^T  |  C(q, e) = tile(q, e)
            if (role <= 2)
                fetch_tile(S, lds, e, p, vc);
            else
                fetch_tile(S, lds, q, e, vc);
        }
        if (role <= 0 && tid < NB) rk[tid] = rhs[(long long)NB * e + tid];
        put_tile(As, va, false);
        if (role > 0) put_tile(Cs, vc, role <= 2);
    }
    __syncthreads();
    const bool ok = block_potrf_inv(As, Bs, false);
    if (role > 0) {
        const int h = (role - 1) & 1;
        d4 acc[2];
        mfma_half(Cs, Bs, h, acc, true);
        __syncthreads();
        half_to_lds(acc, Cs, h, 1.0, false);
        __syncthreads();
        store_rowmajor_half(crL + (long long)NB * NB * (role <= 2 ? e : nt + e), Cs, h);
        return;
    }
    gemv64(Bs, rk, part, y + (long long)NB * e, 1.0);
    store_rowmajor(linv + (long long)NB * NB * e, Bs);
    if (tid == 0 && !ok) status[0] = 1.0;
    if (split) return;
    d4 acc[2][2];
    if (p >= 0) {   // C(p, e) = tile(e, p)^T
        load_tile_t(S, lds, e, p, Cs);
        __syncthreads();
        mfma_64x64(Cs, Bs, acc);
        __syncthreads();
        acc_to_lds(acc, Cs, 1.0, false);
        __syncthreads();
        store_rowmajor(crL + (long long)NB * NB * e, Cs);
        __syncthreads();
    }
    if (q >= 0) {   // C(q, e) = tile(q, e)
        load_tile(S, lds, q, e, Cs);
        __syncthreads();
        mfma_64x64(Cs, Bs, acc);
        __syncthreads();
        acc_to_lds(acc, Cs, 1.0, false);
        __syncthreads();
        store_rowmajor(crL + (long long)NB * NB * (nt + e), Cs);
    }
}

// Update step of a level.  split = 0: one workgroup per kept tile.  split = 1:
// four workgroups per kept tile -- roles 0/1 update rows halves of D_k (role 0
// also r_k), roles 2/3 form rows halves of the fill C(k2, k).
__global__ __launch_bounds__(256) void k_cr_update(double *__restrict__ S, long long lds,
                                                   const int *__restrict__ keep, int nt,
                                                   const double *__restrict__ crL,
                                                   double *__restrict__ rhs,
                                                   const double *__restrict__ y, int split)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP, *Cs = sm + 2 * NB * LP;
    __shared__ double ym[NB], yp[NB], um[NB], up[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x;
    const int x = split ? blockIdx.x >> 2 : blockIdx.x, role = split ? blockIdx.x & 3 : -1;
    const int *kp = keep + 4 * x;
    const int k = kp[0], em = kp[1], ep = kp[2], k2 = kp[3];
    const long long T2 = (long long)NB * NB;
    if (role >= 2) {   // C(k2, k) = -Lq_{e+} Lp_{e+}^T, rows half role - 2
        if (k2 < 0) return;
        const int h = role - 2;
        load_rowmajor(crL + T2 * (nt + ep), Bs);
        load_rowmajor(crL + T2 * ep, Cs);
        __syncthreads();
        d4 acc[2];
        mfma_half(Bs, Cs, h, acc, true);
        half_to_lds(acc, As, h, -1.0, false);
        __syncthreads();
        store_tile_half(S, lds, k2, k, As, h);
        return;
    }
    if (role >= 0) {   // rows half `role` of D_k
        const int h = role;
        load_tile_half(S, lds, k, k, As, h);
        load_rowmajor(crL + T2 * (nt + em), Bs);   // Lq_{e-} = L(k, e-)
        if (ep >= 0) load_rowmajor(crL + T2 * ep, Cs);   // Lp_{e+} = L(k, e+)
        if (h == 0 && tid < NB) {
            ym[tid] = y[(long long)NB * em + tid];
            yp[tid] = (ep >= 0) ? y[(long long)NB * ep + tid] : 0.0;
        }
        __syncthreads();
        d4 acc[2];
        mfma_half(Bs, Bs, h, acc, true);
        if (ep >= 0) mfma_half(Cs, Cs, h, acc, false);
        half_to_lds(acc, As, h, -1.0, true);   // each thread updates the elements it owns
        if (h == 0) {
            gemv64(Bs, ym, part, um, 1.0);
            if (ep >= 0) gemv64(Cs, yp, part, up, 1.0);
            if (tid < NB) {
                double r = rhs[(long long)NB * k + tid] - um[tid];
                if (ep >= 0) r -= up[tid];
                rhs[(long long)NB * k + tid] = r;
            }
        }
        __syncthreads();
        store_tile_half(S, lds, k, k, As, h);
        return;
    }
    load_tile(S, lds, k, k, As);
    load_rowmajor(crL + T2 * (nt + em), Bs);   // Lq_{e-} = L(k, e-)
    if (ep >= 0) load_rowmajor(crL + T2 * ep, Cs);   // Lp_{e+} = L(k, e+)
    if (tid < NB) {
        ym[tid] = y[(long long)NB * em + tid];
        yp[tid] = (ep >= 0) ? y[(long long)NB * ep + tid] : 0.0;
    }
    __syncthreads();
    d4 acc[2][2];
    mfma_64x64(Bs, Bs, acc);
    if (ep >= 0) mfma_64x64_acc(Cs, Cs, acc);
    acc_to_lds(acc, As, -1.0, true);   // each thread updates the elements it owns
    gemv64(Bs, ym, part, um, 1.0);
    if (ep >= 0) gemv64(Cs, yp, part, up, 1.0);
    if (tid < NB) {
        double r = rhs[(long long)NB * k + tid] - um[tid];
        if (ep >= 0) r -= up[tid];
        rhs[(long long)NB * k + tid] = r;
    }
    __syncthreads();
    store_tile(S, lds, k, k, As);
    if (k2 >= 0) {   // C(k2, k) = -Lq_{e+} Lp_{e+}^T
        __syncthreads();
        load_rowmajor(crL + T2 * (nt + ep), Bs);
        __syncthreads();
        mfma_64x64(Bs, Cs, acc);
        __syncthreads();
        acc_to_lds(acc, As, -1.0, false);
        __syncthreads();
        store_tile(S, lds, k2, k, As);
    }
}

// ---------------------------------------------------------------------------
// Camera-aligned cyclic reduction on tiles of TB = NA * floor(32 / NA) rows
// (whole cameras; S rows g = TB * tile + r, r < TB, g < ld).  A tile lives in
// LDS as 32 x 32 (pitch LP, so the 16 x 16 MFMA helpers above apply): rows or
// columns r >= TB, or g >= ld, are padding -- zero, with a unit diagonal in a
// diagonal tile -- so the padded factorisation is that of the TB x TB tile
// bordered by an identity, and padding never leaks into real entries (the
// factors' padding rows / columns are zero off the diagonal).  Same algebra
// and launch structure as the 64-row kernels; the pivot chain per level is
// 32 columns instead of 64.
// ---------------------------------------------------------------------------
#define T32 32

// In-launch hand-offs of the one-launch cyclic reduction (k_cr32_fused):
// every byte one workgroup hands to another is stored write-through (sc1,
// 8-byte agent-scope atomic stores) and every load of it is an sc1 load
// (8-byte agent-scope atomic loads, L1 bypassed), one workgroup per CU, the
// flag an sc1 store after each storing wave's vmcnt(0) and a barrier: the
// first row of MI355X_MICROARCH.md's hand-off table (no acquire fence).
// SC = false: plain accesses (the per-level kernels, whose hand-offs cross a
// launch boundary).
template <bool SC = false>
__device__ __forceinline__ void load32(const double *__restrict__ S, long long lds, int TB,
                                       long long ld, int ti, int tj, double *T, bool transposed,
                                       bool diag)
{
    const int r = threadIdx.x & 31, c0 = threadIdx.x >> 5;
    const long long gr = (long long)TB * ti + r;
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int c = c0 + 8 * u;
        const long long gc = (long long)TB * tj + c;
        const bool ok = r < TB && c < TB && gr < ld && gc < ld;
        v[u] = ok ? ldg<SC>(S + gr + lds * gc) : ((diag && r == c) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int c = c0 + 8 * u;
        if (transposed)
            T[c * LP + r] = v[u];
        else
            T[r * LP + c] = v[u];
    }
}

template <bool SC = false>
__device__ __forceinline__ void store32(double *__restrict__ S, long long lds, int TB,
                                        long long ld, int ti, int tj, const double *T)
{
    const int r = threadIdx.x & 31, c0 = threadIdx.x >> 5;
    const long long gr = (long long)TB * ti + r;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int c = c0 + 8 * u;
        const long long gc = (long long)TB * tj + c;
        if (r < TB && c < TB && gr < ld && gc < ld) stg<SC>(S + gr + lds * gc, T[r * LP + c]);
    }
}

// 32 x 32 LDS tile <-> row-major dst[r * 32 + c]
template <bool SC = false>
__device__ __forceinline__ void store_rm32(double *__restrict__ dst, const double *T)
{
    const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
#pragma unroll
    for (int u = 0; u < 4; u++) stg<SC>(dst + (r0 + 8 * u) * T32 + c, T[(r0 + 8 * u) * LP + c]);
}

template <bool SC = false>
__device__ __forceinline__ void load_rm32(const double *__restrict__ src, double *T)
{
    const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = ldg<SC>(src + (r0 + 8 * u) * T32 + c);
#pragma unroll
    for (int u = 0; u < 4; u++) T[(r0 + 8 * u) * LP + c] = v[u];
}

// One wave's copy of a whole 32 x 32 tile (load32 / load_rm32 with the 256
// threads' elements on the 64 lanes of one wave: the same values at the same
// LDS places), for the level records that wait for each operand's flag in the
// wave that loads it (cr32_level_body's PW form)
__device__ __forceinline__ void load32_wave(const double *__restrict__ S, long long lds, int TB,
                                            long long ld, int ti, int tj, double *T, bool transposed,
                                            bool diag)
{
    const int lane = threadIdx.x & 63, r = lane & 31, c0 = lane >> 5;
    const long long gr = (long long)TB * ti + r;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int c = c0 + 2 * u;
        const long long gc = (long long)TB * tj + c;
        const bool ok = r < TB && c < TB && gr < ld && gc < ld;
        v[u] = ok ? ldg<true>(S + gr + lds * gc) : ((diag && r == c) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int c = c0 + 2 * u;
        if (transposed)
            T[c * LP + r] = v[u];
        else
            T[r * LP + c] = v[u];
    }
}

__device__ __forceinline__ void load_rm32_wave(const double *__restrict__ src, double *T)
{
    const int lane = threadIdx.x & 63, c = lane & 31, r0 = lane >> 5;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = ldg<true>(src + (r0 + 2 * u) * T32 + c);
#pragma unroll
    for (int u = 0; u < 16; u++) T[(r0 + 2 * u) * LP + c] = v[u];
}

// acc (one 16 x 16 block per wave: rows 16 (w >> 1), cols 16 (w & 1)) of
// A B^T over K = 32 (nt form, as mfma_64x64)
__device__ __forceinline__ d4 mfma32_nt(const double *A, const double *Bt, d4 acc)
{
    const int w = threadIdx.x >> 6, ra = 16 * (w >> 1), cb = 16 * (w & 1);
    acc = mfma16_nt(A, ra, 0, Bt, cb, 0, acc);
    return mfma16_nt(A, ra, 16, Bt, cb, 16, acc);
}

__device__ __forceinline__ void put32(double *T, d4 acc, double scale, bool add)
{
    const int w = threadIdx.x >> 6;
    put16(T, 16 * (w >> 1), 16 * (w & 1), acc, scale, add);
}

// out[r] = scale * sum_c M[r][c] v[c] (t = 0) or sum_c M[c][r] v[c] (t = 1),
// r < 32: thread (r, part of 4 columns), the 8 parts added in fixed order
__device__ __forceinline__ void gemv32(const double *M, const double *v, double (*part)[T32],
                                       double *out, bool t)
{
    const int tid = threadIdx.x, r = tid & 31, pq = tid >> 5;
    double acc = 0.0;
#pragma unroll
    for (int c = 4 * pq; c < 4 * pq + 4; c++)
        acc = fma(t ? M[c * LP + r] : M[r * LP + c], v[c], acc);
    part[pq][r] = acc;
    __syncthreads();
    if (tid < T32)
        out[tid] = ((((((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid]) +
                     part[4][tid]) + part[5][tid]) + part[6][tid]) + part[7][tid];
    __syncthreads();
}

// One wave: wave_factor16's Cholesky of the 16x16 diagonal block at (o, o)
// of As, and forward substitutions z = L^-1 v of up to 48 more vectors in
// the same loop.  Every 16-lane row of the wave holds a copy of the factor
// rows (lane l: row l & 15), so each row's DPP broadcasts see the factor's
// column and the copies stay bit-identical; lanes 0..15 carry the identity
// (column r of L^-1 -> Li, if Li), lanes 16 + i (i < 16) vector i of segment
// lo and lanes 32 + i (i < 32) vector i of segment hi (in == nullptr: none).
// The substitutions ride on the factor's broadcasts, so a panel A L^-T (rows
// of A as the vectors) costs no separate stage.  Every lane issues the same
// 16 unconditional LDS loads for its start vector (e_r and zeros from a
// small LDS row), so the loads are in flight together and need no selects.  Lanes 0..15 write L (zero upper) to As.
// Returns false on a non-positive pivot.
struct vseg {
    const double *in;   // entry c of vector i: in[i * irs + c * ics]
    double *out;        // result entry c:      out[i * ors + c * ocs]
    int irs, ics, ors, ocs;
    int n;              // vectors (lanes 16 / 32 + i, i < n)
};

__device__ __forceinline__ bool wave_factor16x(double *As, double *Li, int o, vseg lo, vseg hi)
{
    // e_r for lanes r < 16 and zeros for idle lanes come from one LDS row
    // (ident[16] = 1), so every lane's start vector is one strided read
    __shared__ double ident[33];
    const int lane = threadIdx.x & 63, r = lane & 15;
    if (lane < 33) ident[lane] = lane == 16 ? 1.0 : 0.0;
    const bool up = lane >= 32;
    const int idx = up ? lane - 32 : lane - 16;
    const double *sin = up ? hi.in : lo.in;
    const bool act = lane >= 16 && sin != nullptr && idx < (up ? hi.n : lo.n);
    const double *pin =
        act ? sin + idx * (up ? hi.irs : lo.irs) : (lane < 16 ? ident + 16 - r : ident);
    const int ics = act ? (up ? hi.ics : lo.ics) : 1;
    double d[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) d[c] = As[(o + r) * LP + o + c];
    __builtin_amdgcn_wave_barrier();   // ident written (same wave: LDS in order)
#pragma unroll
    for (int q = 0; q < 16; q++) x[q] = pin[q * ics];
    auto rsq = [&](double piv) {
        double y = __builtin_amdgcn_rsq(piv);
        const double hp = 0.5 * piv;
        y = y * fma(-hp * y, y, 1.5);
        y = y * fma(-hp * y, y, 1.5);
        return y;
    };
    double y = rsq(rowbcast_c<0>(d[0]));
#pragma unroll
    for (int c = 0; c < 16; c++) {
        d[c] = d[c] * y;
        x[c] = x[c] * y;
        if (c + 1 < 16) {
            const double b = rowbcast(d[c], c + 1);
            d[c + 1] = fma(-d[c], b, d[c + 1]);
            y = rsq(rowbcast(d[c + 1], c + 1));
            x[c + 1] = fma(-b, x[c], x[c + 1]);
        }
#pragma unroll
        for (int q = c + 2; q < 16; q++) {
            const double b = rowbcast(d[c], q);
            d[q] = fma(-d[c], b, d[q]);
            x[q] = fma(-b, x[c], x[q]);
        }
#pragma unroll
        for (int q = c; q < 16; q++) asm volatile("" : "+v"(x[q]));
    }
    double dg = 1.0;
#pragma unroll
    for (int c = 0; c < 16; c++)
        if (r == c) dg = d[c];
    const bool ok = __all(lane >= 16 || (dg > 0.0 && dg < __builtin_inf()));
    if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) As[(o + r) * LP + o + c] = (c <= r) ? d[c] : 0.0;
        if (Li) {
#pragma unroll
            for (int c = 0; c < 16; c++) Li[(o + c) * LP + o + r] = x[c];
        }
    } else if (act) {
        double *po = (up ? hi.out : lo.out) + idx * (up ? hi.ors : lo.ors);
        const int ocs = up ? hi.ocs : lo.ocs;
#pragma unroll
        for (int c = 0; c < 16; c++) po[c * ocs] = x[c];
    }
    return ok;
}

// The 32 x 32 Cholesky of As (lower; block (0, 1) keeps A) and, if Li, L^-1
// (row-major, zero upper) -> Li, and, if Cm, the panel Cm L^-T in place (32
// rows), as two wave_factor16x stages with one MFMA stage between them:
//   F0 (wave 0): L00; L10 = A10 L00^-T (lanes 16..31, in place); P0 = C0
//      L00^-T (lanes 32..63, in place) -- or, without a panel and with rv,
//      y0 = L00^-1 r0 (lane 32) -> yv; Li00 (lanes 0..15).  Waves 1..3 run
//      side(w) meanwhile (work F1 needs but F0 does not, e.g. the rest of a
//      pending update of A11 or C1).
//   M: A11 -= L10 L10^T (wave 0); C1 -= P0 L10^T (waves 1, 2) or r1 -= L10
//      y0 (wave 1, in rv); V = -L10 Li00 (wave 3, for Li10).
//   F1 (wave 0): L11; P1 = C1 L11^-T (lanes 32..63) or y1 = L11^-1 r1
//      (lane 32); Li11 (lanes 0..15); Li10 = L11^-1 V (lanes 16..31).
// The critical path is the two 16-pivot chains plus one MFMA stage: the
// panel and the inverse's off-diagonal block need no stage of their own.
// The caller synchronises after filling As / Cm; results visible on return.
#ifdef BA_STAMPS
__device__ unsigned long long g_chst[8192][2];
#define CH_ST(k)                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0 && blockIdx.x < 8192)                                        \
            g_chst[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
extern "C" int vlgba_debug_chstamps(unsigned long long *out, int nrec)
{
    if (nrec > 8192) nrec = 8192;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chst), sizeof(unsigned long long) * 2 * nrec) ==
                   hipSuccess
               ? 0
               : -1;
}
#else
#define CH_ST(k)
#endif

template <class Side>
__device__ __forceinline__ bool cr32_chol(double *As, double *Li, double *Cm, double *Xs,
                                          double *rv, double *yv, Side side)
{
    __shared__ int bad32;
    const int tid = threadIdx.x, w = tid >> 6;
    if (Li) Li[(tid >> 4) * LP + 16 + (tid & 15)] = 0.0;   // block (0, 1) of L^-1
    if (w == 0) {
        const vseg lo{As + 16 * LP, As + 16 * LP, LP, 1, LP, 1, 16};   // A10 rows -> L10
        const vseg hi = Cm ? vseg{Cm, Cm, LP, 1, LP, 1, 32}            // C0 rows -> P0
                           : vseg{rv, yv, 0, 1, 0, 1, 1};              // or r0 -> y0
        const bool ok = wave_factor16x(As, Li, 0, lo, hi);
        if (tid == 0) bad32 = ok ? 0 : 1;
    } else {
        side(w);
    }
    __syncthreads();
    CH_ST(0);
    if (w == 0) {   // A11 -= L10 L10^T
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nt(As, 16, 0, As, 16, 0, acc);
        put16(As, 16, 16, acc, -1.0, true);
    } else if (w <= 2) {   // C1 -= P0 L10^T, rows 16 (w - 1) ..
        if (Cm) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma16_nt(Cm, 16 * (w - 1), 0, As, 16, 0, acc);
            put16(Cm, 16 * (w - 1), 16, acc, -1.0, true);
        } else if (rv && w == 1 && (tid & 63) < 16) {   // r1' = r1 - L10 y0
            const int r = tid & 63;
            double t = 0.0;
#pragma unroll
            for (int c = 0; c < 16; c++) t = fma(As[(16 + r) * LP + c], yv[c], t);
            rv[16 + r] = rv[16 + r] - t;
        }
    } else if (Li) {   // V = -L10 Li00
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nn(As, 16, 0, Li, 0, 0, acc);
        put16(Xs, 0, 0, acc, -1.0, false);
    }
    __syncthreads();
    CH_ST(1);
    if (w == 0) {
        // V's columns -> Li10's columns; C1 rows -> P1, or r1' -> y1
        const vseg lo{Li ? Xs : nullptr, Li ? Li + 16 * LP : nullptr, 1, LP, 1, LP, 16};
        const vseg hi = Cm ? vseg{Cm + 16, Cm + 16, LP, 1, LP, 1, 32}
                           : vseg{rv ? rv + 16 : nullptr, yv ? yv + 16 : nullptr, 0, 1, 0, 1, 1};
        const bool ok = wave_factor16x(As, Li, 16, lo, hi);
        if (tid == 0 && !ok) bad32 = 1;
    }
    __syncthreads();
    return bad32 == 0;
}

// The envelope's 64 x 64 diagonal factor and L^-1 (row-major, zero upper, in
// Bs) as two cr32_chol factors: F(A00) -> L00, Li00 and the panel L10 = A10
// L00^-T on the same pivot chains; then A11 -= L10 L10^T (waves 0-2, its
// three lower 16-blocks) beside T = L10 Li00 (into Bs's block (1, 0)); F(A11)
// -> L11, Li11; Li10 = -Li11 T.  Two 32-row factors (~8.2k cycles each,
// profiles/r04c_ubench_cr32.txt) instead of four dependent 16-row stages with
// their updates in between (block_potrf_inv, ~29.5k cycles).  Xs: 16 x LP
// scratch.  Ends with a barrier.
__device__ __forceinline__ bool potrf64_via32(double *As, double *Bs, double *Xs)
{
    const int tid = threadIdx.x, w = tid >> 6;
    for (int q = tid; q < 32 * 32; q += blockDim.x) Bs[(q >> 5) * LP + 32 + (q & 31)] = 0.0;
    bool ok = cr32_chol(As, Bs, As + 32 * LP, Xs, nullptr, nullptr, [](int) {});
    {
        // A11 -= L10 L10^T: blocks (32, 32), (48, 32), (48, 48) by waves 0..2;
        // T = L10 Li00 blocks (32 + 16 (u >> 1), 16 (u & 1)), u = w and w + 4 - 1 ...
        const int ri = w == 0 ? 32 : 48, ci = w == 2 ? 48 : 32;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        if (w < 3) {
            acc = mfma16_nt(As, ri, 0, As, ci, 0, acc);
            acc = mfma16_nt(As, ri, 16, As, ci, 16, acc);
        }
        // T blocks: wave 3 takes (32, 0) and (32, 16), waves 0 / 1 take (48, 0) / (48, 16)
        d4 t0 = {0.0, 0.0, 0.0, 0.0}, t1 = {0.0, 0.0, 0.0, 0.0};
        if (w == 3) {
            t0 = mfma16_nn(As, 32, 0, Bs, 0, 0, t0);
            t0 = mfma16_nn(As, 32, 16, Bs, 16, 0, t0);
            t1 = mfma16_nn(As, 32, 16, Bs, 16, 16, t1);   // Li00 block (0, 1) is zero
        } else if (w < 2) {
            t0 = mfma16_nn(As, 48, 0, Bs, 0, 16 * w, t0);
            t0 = mfma16_nn(As, 48, 16, Bs, 16, 16 * w, t0);
        }
        if (w < 3) put16(As, ri, ci, acc, -1.0, true);
        if (w == 3) {
            put16(Bs, 32, 0, t0, 1.0, false);
            put16(Bs, 32, 16, t1, 1.0, false);
        } else if (w < 2) {
            put16(Bs, 48, 16 * w, t0, 1.0, false);
        }
    }
    __syncthreads();
    ok = cr32_chol(As + 32 * LP + 32, Bs + 32 * LP + 32, nullptr, Xs, nullptr, nullptr,
                   [](int) {}) && ok;
    {   // Li10 = -Li11 T, block (32 + 16 (w >> 1), 16 (w & 1)) by wave w
        const int ri = 32 + 16 * (w >> 1), cj = 16 * (w & 1);
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nn(Bs, ri, 32, Bs, 32, cj, acc);
        acc = mfma16_nn(Bs, ri, 48, Bs, 48, cj, acc);
        __syncthreads();
        put16(Bs, ri, cj, acc, -1.0, false);
    }
    __syncthreads();
    return ok;
}

// LDS of one cyclic-reduction record: five 32-row tiles, the 16-row scratch
// of potrf32_inv, five 32-vectors and the gemv partials.  The per-level
// kernels declare it as static LDS; k_cr32_fused carves every record type
// (factor, fused level, survivor, back substitution) from one pool of this
// shape (96 KB: one workgroup per CU, which its hand-offs rely on).
struct cr32_lds {
    double *As, *Bs, *Cs, *Ds, *Es, *Xs;
    double *rk, *ym, *yp, *um, *up;
    double (*part)[T32];
};

#define CR32_LDS_DECL                                                                      \
    __shared__ __attribute__((aligned(16))) double cr_As[T32 * LP], cr_Bs[T32 * LP],      \
        cr_Cs[T32 * LP], cr_Ds[T32 * LP], cr_Es[T32 * LP];                                 \
    __shared__ __attribute__((aligned(16))) double cr_Xs[16 * LP];                         \
    __shared__ __attribute__((aligned(16))) double cr_v[5][T32];                           \
    __shared__ __attribute__((aligned(16))) double cr_part[8][T32];                        \
    const cr32_lds sh{cr_As, cr_Bs, cr_Cs, cr_Ds, cr_Es, cr_Xs, cr_v[0], cr_v[1], cr_v[2], \
                      cr_v[3], cr_v[4], cr_part}

// Diagnostic build only (make stamps): per record of k_cr32_fused, the
// s_memrealtime (100 MHz) at entry, after its wait, before and after its
// publish, and inside the record bodies (SC instantiation only): [4] loads
// in LDS, [5] update applied, [6] factor + panel done, [7] before the panel
// store; [8] / [9] cr32_chol's first pivot chain / MFMA stage done
// (tools/cr_timeline.py)
#ifdef BA_STAMPS
#define CR_ST_MAX 8192
__device__ unsigned long long g_crst[CR_ST_MAX][12];
extern "C" int vlgba_debug_crstamps(unsigned long long *out, int nrec)
{
    if (nrec > CR_ST_MAX) nrec = CR_ST_MAX;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_crst), sizeof(unsigned long long) * 12 * nrec) ==
                   hipSuccess
               ? 0
               : -1;
}
#define CR_ST(k)                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0 && blockIdx.x < CR_ST_MAX)                                   \
            g_crst[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
#define CR_SUB(k)                                                                         \
    do {                                                                                  \
        if constexpr (SC)                                                                 \
            if (threadIdx.x == 0 && blockIdx.x < CR_ST_MAX)                               \
                g_crst[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                 \
    } while (0)
#else
#define CR_ST(k)
#define CR_SUB(k)
#endif

// factor step (level 0, on the assembled S): role 0 factors D_e, writes L_e^-1
// (row-major 32 x 32) and y_e = L_e^-1 r_e; role 1 / 2 (split, one workgroup
// each, redoing the same factorisation) form Lp_e = C(p, e) L_e^-T / Lq_e =
// C(q, e) L_e^-T into crL (the panel rides on the factor: cr32_chol); role 4
// = roles 0 and 1 in one workgroup (y by a GEMV with L^-1 there: the panel
// takes the factor's spare lanes); role -1 (no split) = role 4, then the
// factorisation again for the q panel (the same operations as role 2, so the
// split and unsplit launches agree bit for bit).
template <bool SC>
__device__ __forceinline__ void cr32_factor_body(const cr32_lds &sh, double *S, long long lds,
                                                 int TB, long long ld, int e, int p, int q,
                                                 int role, int nt, double *linv, double *crL,
                                                 const double *rhs, double *y, double *status)
{
    double *As = sh.As, *Bs = sh.Bs, *Cs = sh.Cs, *Xs = sh.Xs, *rk = sh.rk, *yk = sh.ym;
    const int tid = threadIdx.x;
    const long long T2 = (long long)T32 * T32;
    const bool rows = role <= 0 || role == 4;
    const int side = role == 2 ? 2 : 1;   // the panel of this pass (role 0: none)
    const bool pan = (role == 1 || role == 4 || role < 0) ? p >= 0 : (role == 2 && q >= 0);
    load32<SC>(S, lds, TB, ld, e, e, As, false, true);
    if (pan && side == 1) load32<SC>(S, lds, TB, ld, e, p, Cs, true, false);   // C(p, e) = tile(e, p)^T
    if (pan && side == 2) load32<SC>(S, lds, TB, ld, q, e, Cs, false, false);  // C(q, e) = tile(q, e)
    if (rows && tid < T32) {
        const long long g = (long long)TB * e + tid;
        rk[tid] = (tid < TB && g < ld) ? ldg<SC>(rhs + g) : 0.0;
    }
    __syncthreads();
    CR_SUB(4);
    CR_SUB(5);
    // y rides on the factor's spare lanes unless a panel fills them (roles 4, -1)
    const bool ylanes = rows && !pan;
    const bool ok = cr32_chol(As, rows ? Bs : nullptr, pan ? Cs : nullptr, Xs,
                              ylanes ? rk : nullptr, yk, [](int) {});
    CR_SUB(6);
    if (pan) {
        CR_SUB(7);
        store_rm32<SC>(crL + T2 * (side == 1 ? e : nt + e), Cs);
    }
    if (rows) {
        if (!ylanes) gemv32(Bs, rk, sh.part, yk, false);
        if (tid < TB) stg<SC>(y + (long long)TB * e + tid, yk[tid]);
        store_rm32<SC>(linv + T2 * e, Bs);
        if (tid == 0 && !ok) status[0] = 1.0;
    }
    if (role < 0 && q >= 0) {   // unsplit: the q panel (role 2's pass)
        __syncthreads();
        load32<SC>(S, lds, TB, ld, e, e, As, false, true);
        load32<SC>(S, lds, TB, ld, q, e, Cs, false, false);
        __syncthreads();
        cr32_chol(As, nullptr, Cs, Xs, nullptr, nullptr, [](int) {});
        store_rm32<SC>(crL + T2 * (nt + e), Cs);
    }
}

__global__ __launch_bounds__(256) void k_cr32_factor(double *__restrict__ S, long long lds,
                                                     int TB, long long ld,
                                                     const int *__restrict__ elim, int nt,
                                                     double *__restrict__ linv,
                                                     double *__restrict__ crL,
                                                     const double *__restrict__ rhs,
                                                     double *__restrict__ y,
                                                     double *__restrict__ status, int split)
{
    __shared__ __attribute__((aligned(16))) double As[T32 * LP], Bs[T32 * LP], Cs[T32 * LP];
    __shared__ __attribute__((aligned(16))) double Xs[16 * LP];
    __shared__ double rk[T32], yk[T32];
    __shared__ double part[8][T32];
    const cr32_lds sh{As, Bs, Cs, nullptr, nullptr, Xs, rk, yk, nullptr, nullptr, nullptr, part};
    const int x = split ? blockIdx.x / 3 : blockIdx.x, role = split ? blockIdx.x % 3 : -1;
    const int e = elim[3 * x], p = elim[3 * x + 1], q = elim[3 * x + 2];
    if ((role == 1 && p < 0) || (role == 2 && q < 0)) return;
    cr32_factor_body<false>(sh, S, lds, TB, ld, e, p, q, role, nt, linv, crL, rhs, y, status);
}

// Level L >= 1 of the camera-aligned CR with the previous level's update folded
// in (one launch per level instead of two).  Tile k of level L carries the
// update of level L-1,
//     D_k -= L(k, em) L(k, em)^T + L(k, ep) L(k, ep)^T,  r_k -= L(k, em) y_em + L(k, ep) y_ep
// (em / ep: the tiles eliminated at L-1 next to k), and the coupling of two
// neighbours k < k2 at level L is the fill C(k2, k) = -L(k2, e) L(k, e)^T of
// the tile e eliminated between them.  Workgroups 3x + role for the tiles
// eliminated here (role 0: apply the update, factor, y, L^-1; roles 1 / 2:
// the same factorisation with their fill tile C(p, e) / C(q, e) as the panel
// rows of cr32_chol), then one workgroup per surviving tile (role 3: apply
// the update, write D_k back, mid(), then r_k).  Records: fused (e, p, q,
// em, ep), survivor (k, em, ep).  The eliminated tiles' update is split by
// 16 x 16 block: D00 and D10 (and the fill's first 16 columns) before the
// first pivot chain, D11 and the rest of the fill beside it (cr32_chol's
// side); role 0's r update runs beside the D00 / D10 blocks.  mid: the
// survivor's D_k is published before its r_k (k_cr32_fused: the panel roles
// of the next level need only D_k, and r_k waits for the neighbours' y).
// r_k -= L(k, em) y_em + L(k, ep) y_ep by one wave: lane r < 32 row r of the
// first product, lane 32 + r of the second, each a sequential sum over the
// 32 columns.
__device__ __forceinline__ void cr32_rupd(const double *Bs, const double *Cs, bool two,
                                          const double *ym, const double *yp, double *rk,
                                          double *up)
{
    const int lane = threadIdx.x & 63, r = lane & 31;
    const double *M = lane < 32 ? Bs : Cs;
    const double *v = lane < 32 ? ym : yp;
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < T32; c++) t = fma(M[r * LP + c], v[c], t);
    if (lane >= 32) up[r] = two ? t : 0.0;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < 32) rk[r] = (rk[r] - t) - up[r];
}

// The one-launch CR's per-wave operand hand-off (k_cr32_fused, level L >= 1):
// each wave polls only the flags of the operand it loads and loads it at once
// (all 64 lanes, sc1), so an operand whose producer finished early is in LDS
// while the wave of a later one still waits; one barrier after all of them.
// The union of the waves' flags is the record's former flag set.
struct cr32_pw {
    const unsigned *flag;
    unsigned epoch;
    double *status;
    int L, nt;
};

__device__ __forceinline__ void cr32_wave_wait(const cr32_pw &pw, const int *w, int nw)
{
    const int lane = threadIdx.x & 63;
    int idx = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (lane == q && q < nw) idx = w[q];
    for (unsigned spins = 0;; spins++) {
        const bool ok = lane >= nw || __hip_atomic_load((const gu32_t *)(pw.flag + idx),
                                                        __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) == pw.epoch;
        if (__all(ok)) break;
        if (spins >= BA_BACK_SPIN_MAX) {
            if (lane == 0) pw.status[1] = 1.0;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <bool SC, class Mid>
__device__ __forceinline__ void cr32_level_body(const cr32_lds &sh, double *S, long long lds,
                                                int TB, long long ld, int k, int p, int q, int em,
                                                int ep, int role, int nt, double *linv,
                                                double *crL, double *rhs, double *y,
                                                double *status, Mid mid,
                                                const cr32_pw *pw = nullptr)
{
    double *As = sh.As, *Bs = sh.Bs, *Cs = sh.Cs, *Ds = sh.Ds, *Es = sh.Es, *Xs = sh.Xs;
    double *rk = sh.rk, *ym = sh.ym, *yp = sh.yp, *um = sh.um, *up = sh.up;
    const int tid = threadIdx.x, w = tid >> 6;
    const long long T2 = (long long)T32 * T32;
    const bool surv = role == 3;
    auto load_r = [&]() {
        if (tid < T32) {
            const long long g = (long long)TB * k + tid;
            rk[tid] = (tid < TB && g < ld) ? ldg<SC>(rhs + g) : 0.0;
            ym[tid] = tid < TB ? ldg<SC>(y + (long long)TB * em + tid) : 0.0;
            yp[tid] = (ep >= 0 && tid < TB) ? ldg<SC>(y + (long long)TB * ep + tid) : 0.0;
        }
    };
    if (SC && pw) {   // per wave: its operand's flags, then its operand
        auto fw = [&](int t, int r) { return 5 * ((pw->L - 1) * nt + t) + r; };
        const bool own = pw->L >= 2;
        int wl[4], n = 0;
        if (w == 0) {          // D_k (its survivor record at L - 1)
            if (own) {
                wl[n++] = fw(k, 3);
                if (role == 0) wl[n++] = fw(k, 4);
            }
            cr32_wave_wait(*pw, wl, n);
            load32_wave(S, lds, TB, ld, k, k, As, false, true);
        } else if (w == 1) {   // L(k, em) = role 2 of em (role 0 waits for all of em)
            wl[n++] = fw(em, 2);
            if (role == 0 || role == 1) wl[n++] = fw(em, 1);
            if (role == 0) wl[n++] = fw(em, 0);
            cr32_wave_wait(*pw, wl, n);
            load_rm32_wave(crL + T2 * (nt + em), Bs);
        } else if (w == 2) {   // L(k, ep) = role 1 of ep
            if (ep >= 0) {
                wl[n++] = fw(ep, 1);
                if (role == 0 || role == 2) wl[n++] = fw(ep, 2);
                if (role == 0) wl[n++] = fw(ep, 0);
                cr32_wave_wait(*pw, wl, n);
                load_rm32_wave(crL + T2 * ep, Cs);
            }
        } else if (role == 1 || role == 2) {   // the fill's L(p, em) | L(q, ep)
            wl[n++] = role == 1 ? fw(em, 1) : fw(ep, 2);
            cr32_wave_wait(*pw, wl, n);
            load_rm32_wave(crL + T2 * (role == 1 ? em : nt + ep), Ds);
        } else if (role == 0) {   // r_k, y_em, y_ep on this wave's first 32 lanes
            wl[n++] = fw(em, 0);
            if (ep >= 0) wl[n++] = fw(ep, 0);
            if (own) wl[n++] = fw(k, 4);
            cr32_wave_wait(*pw, wl, n);
            const int i = tid & 63;
            if (i < T32) {
                const long long g = (long long)TB * k + i;
                rk[i] = (i < TB && g < ld) ? ldg<SC>(rhs + g) : 0.0;
                ym[i] = i < TB ? ldg<SC>(y + (long long)TB * em + i) : 0.0;
                yp[i] = (ep >= 0 && i < TB) ? ldg<SC>(y + (long long)TB * ep + i) : 0.0;
            }
        }
        __syncthreads();
    } else {
        load32<SC>(S, lds, TB, ld, k, k, As, false, true);
        load_rm32<SC>(crL + T2 * (nt + em), Bs);            // L(k, em)
        if (ep >= 0) load_rm32<SC>(crL + T2 * ep, Cs);      // L(k, ep)
        if (role == 1) load_rm32<SC>(crL + T2 * em, Ds);    // L(p, em)
        if (role == 2) load_rm32<SC>(crL + T2 * (nt + ep), Ds);   // L(q, ep)
        if (role == 0) load_r();
        __syncthreads();
    }
    CR_SUB(4);
    if (surv) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma32_nt(Bs, Bs, acc);
        if (ep >= 0) acc = mfma32_nt(Cs, Cs, acc);
        put32(As, acc, -1.0, true);   // each thread updates the elements it owns
        __syncthreads();
        store32<SC>(S, lds, TB, ld, k, k, As);
        mid();
        load_r();
        __syncthreads();
        if (w == 0) cr32_rupd(Bs, Cs, ep >= 0, ym, yp, rk, up);
        __syncthreads();
        if (tid < TB) {
            const long long g = (long long)TB * k + tid;
            if (g < ld) stg<SC>(rhs + g, rk[tid]);
        }
        return;
    }
    const double *G = role == 2 ? Cs : Bs;   // the fill's right factor: L(k, em) | L(k, ep)
    // block (ri, ci) of D -= Lm Lm^T + Lp Lp^T (K = 32 each)
    auto dupd = [&](int ri, int ci) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nt(Bs, ri, 0, Bs, ci, 0, acc);
        acc = mfma16_nt(Bs, ri, 16, Bs, ci, 16, acc);
        if (ep >= 0) {
            acc = mfma16_nt(Cs, ri, 0, Cs, ci, 0, acc);
            acc = mfma16_nt(Cs, ri, 16, Cs, ci, 16, acc);
        }
        put16(As, ri, ci, acc, -1.0, true);
    };
    // block (ri, ci) of the fill: Es = -Ds G^T
    auto fill = [&](int ri, int ci) {
        d4 f = {0.0, 0.0, 0.0, 0.0};
        f = mfma16_nt(Ds, ri, 0, G, ci, 0, f);
        f = mfma16_nt(Ds, ri, 16, G, ci, 16, f);
        put16(Es, ri, ci, f, -1.0, false);
    };
    const bool pan = role != 0;
    if (w == 0)
        dupd(0, 0);
    else if (w == 1)
        dupd(16, 0);
    else if (pan)
        fill(16 * (w - 2), 0);
    else if (w == 2)
        cr32_rupd(Bs, Cs, ep >= 0, ym, yp, rk, up);
    __syncthreads();
    CR_SUB(5);
    const bool ok = cr32_chol(As, pan ? nullptr : Ds, pan ? Es : nullptr, Xs, pan ? nullptr : rk,
                              um, [&](int ww) {
                                  if (ww == 1)
                                      dupd(16, 16);
                                  else if (pan)
                                      fill(16 * (ww - 2), 16);
                              });
    CR_SUB(6);
    if (role == 0) {   // L^-1 in Ds (no fill for role 0), y in um
        if (tid < TB) stg<SC>(y + (long long)TB * k + tid, um[tid]);
        store_rm32<SC>(linv + T2 * k, Ds);
        if (tid == 0 && !ok) status[0] = 1.0;
        return;
    }
    CR_SUB(7);
    store_rm32<SC>(crL + T2 * (role == 1 ? k : nt + k), Es);
}

__global__ __launch_bounds__(256) void k_cr32_level(double *__restrict__ S, long long lds, int TB,
                                                    long long ld, const int *__restrict__ frec,
                                                    int ne, const int *__restrict__ srec, int nt,
                                                    double *__restrict__ linv,
                                                    double *__restrict__ crL,
                                                    double *__restrict__ rhs,
                                                    double *__restrict__ y,
                                                    double *__restrict__ status)
{
    CR32_LDS_DECL;
    const bool surv = (int)blockIdx.x >= 3 * ne;
    int k, p = -1, q = -1, em, ep, role = 3;
    if (surv) {
        const int *r = srec + 3 * (blockIdx.x - 3 * ne);
        k = r[0];
        em = r[1];
        ep = r[2];
    } else {
        const int *r = frec + 5 * (blockIdx.x / 3);
        role = blockIdx.x % 3;
        k = r[0];
        p = r[1];
        q = r[2];
        em = r[3];
        ep = r[4];
        if ((role == 1 && p < 0) || (role == 2 && q < 0)) return;
    }
    cr32_level_body<false>(sh, S, lds, TB, ld, k, p, q, em, ep, role, nt, linv, crL, rhs, y,
                           status, [] {});
}

// Back substitution of one eliminated tile e (neighbours p, q):
//     x_e = L_e^-T (y_e - Lp_e^T x_p - Lq_e^T x_q) = z_e - Mp x_p - Mq x_q,
//     z_e = L_e^-T y_e,  Mp = L_e^-T Lp_e^T,  Mq = L_e^-T Lq_e^T.
// z, Mp and Mq need only the factor step's outputs, so they are formed
// before the neighbours' x is fetched (while k_cr32_fused / k_cr32_back_all
// wait for it); after the fetch a single 32 x 64 matrix-vector product
// remains.  fetch(xp, xq) puts x_p / x_q (zero where absent) in LDS and ends
// with a barrier; the caller's loads of the tiles are done and synchronised.
// Mp / Mq overwrite Lp / Lq.  Returns x_e in u.
__device__ __forceinline__ d4 mfma32_tn(const double *At, const double *Bt, d4 acc)
{
    // acc (one 16 x 16 block per wave) of A B^T over K = 32, A given
    // transposed (At[t][r]): [r][c] = sum_t At[t][r] Bt[c][t]
    const int w = threadIdx.x >> 6, ra = 16 * (w >> 1), cb = 16 * (w & 1);
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 8; s++)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(At[(4 * s + lk) * LP + ra + li],
                                                   Bt[(cb + li) * LP + 4 * s + lk], acc, 0, 0, 0);
    return acc;
}

template <class Fetch>
__device__ __forceinline__ void cr32_back_core(double *Lp, double *Lq, const double *Li,
                                               const double *t, double *z, double *xp,
                                               double *xq, double *u, double (*part)[T32],
                                               bool hp, bool hq, Fetch fetch)
{
    const int tid = threadIdx.x;
    d4 ap = {0.0, 0.0, 0.0, 0.0}, aq = {0.0, 0.0, 0.0, 0.0};
    if (hp) ap = mfma32_tn(Li, Lp, ap);   // Mp[r][c] = sum_t Li[t][r] Lp[c][t]
    if (hq) aq = mfma32_tn(Li, Lq, aq);
    gemv32(Li, t, part, z, true);         // z = L^-T y (ends with a barrier)
    if (hp) put32(Lp, ap, 1.0, false);
    if (hq) put32(Lq, aq, 1.0, false);
    fetch(xp, xq);                        // ends with a barrier
    // x = z - [Mp | Mq] [x_p; x_q]: thread (row r, part of 8 columns)
    const int r = tid & 31, pq = tid >> 5;
    const double *M = pq < 4 ? Lp : Lq;
    const double *v = pq < 4 ? xp : xq;
    const bool on = pq < 4 ? hp : hq;
    const int c0 = 8 * (pq & 3);
    double acc = 0.0;
    if (on) {
#pragma unroll
        for (int c = c0; c < c0 + 8; c++) acc = fma(M[r * LP + c], v[c], acc);
    }
    part[pq][r] = acc;
    __syncthreads();
    if (tid < T32)
        u[tid] = z[tid] - ((((((((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid]) +
                               part[4][tid]) + part[5][tid]) + part[6][tid]) + part[7][tid]));
    __syncthreads();
}

// back substitution, one launch per level (the no-spin re-solve): x_p and x_q
// come from the previous launches
__global__ __launch_bounds__(256) void k_cr32_back(const int *__restrict__ elim, int nt, int TB,
                                                   long long ld,
                                                   const double *__restrict__ linv,
                                                   const double *__restrict__ crL,
                                                   const double *__restrict__ y,
                                                   double *__restrict__ x)
{
    __shared__ __attribute__((aligned(16))) double Lp[T32 * LP], Lq[T32 * LP], Li[T32 * LP];
    __shared__ __attribute__((aligned(16))) double t[T32], z[T32], xp[T32], xq[T32], u[T32];
    __shared__ double part[8][T32];
    const int tid = threadIdx.x;
    const int e = elim[3 * blockIdx.x], p = elim[3 * blockIdx.x + 1], q = elim[3 * blockIdx.x + 2];
    const long long T2 = (long long)T32 * T32;
    if (p >= 0) load_rm32(crL + T2 * e, Lp);
    if (q >= 0) load_rm32(crL + T2 * (nt + e), Lq);
    load_rm32(linv + T2 * e, Li);
    if (tid < T32) t[tid] = tid < TB ? y[(long long)TB * e + tid] : 0.0;
    __syncthreads();
    cr32_back_core(Lp, Lq, Li, t, z, xp, xq, u, part, p >= 0, q >= 0,
                   [&](double *a, double *b) {
                       if (tid < 2 * T32) {
                           const int nb = tid < T32 ? p : q, i = tid & 31;
                           const long long g = (long long)TB * nb + i;
                           (tid < T32 ? a : b)[i] = (nb >= 0 && i < TB && g < ld) ? x[g] : 0.0;
                       }
                       __syncthreads();
                   });
    if (tid < TB) {
        const long long g = (long long)TB * e + tid;
        if (g < ld) x[g] = u[tid];
    }
}

// One record of the one-launch back substitution: it loads its three tiles,
// forms z, Mp and Mq (cr32_back_core), then waits for x_p and x_q, which the
// records of the tiles eliminated above it publish as epoch-tagged 8-byte
// granules {epoch, 32-bit half} (write-through agent-scope stores: the data
// is the flag, no fences; MI355X_MICROARCH.md / cdna_hip_programming.md
// Guideline 16, R2).  One wave sweeps one neighbour's 64 granules until every
// tag matches; a spin that never ends sets the timeout word status[1] (the
// host then re-solves the pass with the per-level launches, which never spin)
// instead of hanging.  Same arithmetic as k_cr32_back.
template <bool SC>
__device__ __forceinline__ void cr32_back_body(const cr32_lds &sh, int e, int p, int q, int nt,
                                               int TB, long long ld, const double *linv,
                                               const double *crL, const double *y, double *x,
                                               unsigned long long *xg, unsigned epoch,
                                               double *status)
{
    double *Lp = sh.As, *Lq = sh.Bs, *Li = sh.Cs;
    double *t = sh.rk, *xp = sh.ym, *xq = sh.yp, *u = sh.um, *z = sh.up;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long T2 = (long long)T32 * T32;
    if (p >= 0) load_rm32<SC>(crL + T2 * e, Lp);
    if (q >= 0) load_rm32<SC>(crL + T2 * (nt + e), Lq);
    load_rm32<SC>(linv + T2 * e, Li);
    if (tid < T32) t[tid] = tid < TB ? ldg<SC>(y + (long long)TB * e + tid) : 0.0;
    __syncthreads();
    cr32_back_core(Lp, Lq, Li, t, z, xp, xq, u, sh.part, p >= 0, q >= 0,
                   [&](double *a, double *b) {
                       if (wv < 2) {
                           const int nb = wv == 0 ? p : q;
                           double *dst = wv == 0 ? a : b;
                           if (nb >= 0) {
                               const unsigned long long *g = xg + 64 * (size_t)nb + lane;
                               unsigned long long v = 0;
                               for (unsigned spins = 0;; spins++) {
                                   v = __hip_atomic_load(g, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                                   if (__all((unsigned)(v >> 32) == epoch)) break;
                                   if (spins >= BA_BACK_SPIN_MAX) {
                                       if (lane == 0) status[1] = 1.0;
                                       break;
                                   }
                                   __builtin_amdgcn_s_sleep(2);
                               }
                               // lane 2r: low half of x_r, lane 2r + 1: high half
                               reinterpret_cast<unsigned *>(dst)[lane] = (unsigned)v;
                           } else if (lane < T32) {
                               dst[lane] = 0.0;
                           }
                       }
                       __syncthreads();
                   });
    if (wv == 0) {   // publish x_e: 64 granules, one 8-byte write-through store each
        const unsigned h = reinterpret_cast<const unsigned *>(u)[lane];
        __hip_atomic_store(xg + 64 * (size_t)e + lane, ((unsigned long long)epoch << 32) | h,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < TB) {
        const long long g = (long long)TB * e + tid;
        if (g < ld) x[g] = u[tid];
    }
}

// All levels of the back substitution in ONE launch (the
// 8 level launches were at the launch floor).  Workgroup b takes elimination
// record nrec-1-b (the deepest level first).  Every record's neighbours are
// eliminated at higher levels, so the dependencies form a tree from the top
// level down; the launch is used only when all workgroups are co-resident
// (nrec <= 2 x CUs).
__global__ __launch_bounds__(256) void k_cr32_back_all(const int *__restrict__ elim, int nrec,
                                                       int nt, int TB, long long ld,
                                                       const double *__restrict__ linv,
                                                       const double *__restrict__ crL,
                                                       const double *__restrict__ y,
                                                       double *__restrict__ x,
                                                       unsigned long long *__restrict__ xg,
                                                       unsigned epoch, double *status)
{
    __shared__ __attribute__((aligned(16))) double Lp[T32 * LP], Lq[T32 * LP], Li[T32 * LP];
    __shared__ __attribute__((aligned(16))) double t[T32], xp[T32], xq[T32], u[T32], z[T32];
    __shared__ double part[8][T32];
    const cr32_lds sh{Lp, Lq, Li, nullptr, nullptr, nullptr, t, xp, xq, u, z, part};
    const int rec = nrec - 1 - (int)blockIdx.x;
    const int e = elim[3 * rec], p = elim[3 * rec + 1], q = elim[3 * rec + 2];
    cr32_back_body<false>(sh, e, p, q, nt, TB, ld, linv, crL, y, x, xg, epoch, status);
}

// ---------------------------------------------------------------------------
// The whole camera-aligned cyclic reduction in ONE launch: the level-0
// factor records (3 per eliminated tile), then per level L >= 1 the fused
// records (3 per eliminated tile) and the survivor records, then the back
// substitution records deepest level first -- the schedule and arithmetic of
// k_cr32_factor + k_cr32_level x (nl - 1) + k_cr32_back_all, record for record
// (bit-identical), with the launch boundaries replaced by per-record
// dependencies: a record waits only for the records whose outputs it reads,
//   level L >= 1, tile k (neighbours em / ep eliminated at L-1):
//     role 0 / survivor: roles 0..2 of em and ep at L-1 (L(k, em), L(k, ep),
//     y); roles 1 / 2: only the panels they read (L(k, em) = role 2 of em,
//     L(k, ep) = role 1 of ep, the fill's L(p, em) = role 1 of em or
//     L(q, ep) = role 2 of ep); all: k's own survivor record at L-1 (D_k,
//     r_k) when L >= 2 (survivor records publish D_k and r_k separately: the
//     panel roles wait for D_k only, role 0 for both);
//   survivor at L: L(k, em), L(k, ep) (and D_k at L-1) for D_k, then the
//     neighbours' role 0 (y) and its own r_k at L-1 for r_k;
//   back record of e (eliminated at Le): roles 0..2 of e at Le, then the
//     x granules of its neighbours (as k_cr32_back_all).
// Hand-offs: payload stored sc1 (stg<true>), every storing wave's vmcnt(0),
// a barrier, one lane's sc1 flag store {epoch} per (level, tile, role); the
// consumer's wave 0 polls its <= 7 flags (relaxed agent loads), a barrier,
// then sc1 loads (ldg<true>) of every handed-off byte.  The 96 KB LDS pool
// keeps one workgroup per CU (the row of MI355X_MICROARCH.md's hand-off table
// this protocol follows).  Records wait only on records with lower block
// indices, so in-order dispatch makes progress without co-residency; every
// spin is bounded (timeout word status[1]: the host re-solves with the per-level
// launches).
// ---------------------------------------------------------------------------
#define BA_CR_MAXLEV 30
#ifndef BA_CR_PW
#define BA_CR_PW 1
#endif
struct cr32_fplan {
    int nl, nrec;
    int l0two;                     // level 0 in 2 records per tile (roles 4 | 2), else 3
    int b0[BA_CR_MAXLEV + 2];      // first block of level L; b0[nl] = first back block
    int fofs[BA_CR_MAXLEV + 1];    // level L >= 1: first fused record in crf
    int sofs[BA_CR_MAXLEV + 1];    //               first survivor record in crs
    int eofs[BA_CR_MAXLEV + 2];    // elimination records of level L in cr_elim
};

__device__ __forceinline__ void cr32_wait_flags(const unsigned *flag, int nw, const int w[8],
                                                unsigned epoch, double *status)
{
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int idx = 0;
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (lane == q) idx = w[q];
        for (unsigned spins = 0;; spins++) {
            const bool ok = lane >= nw || __hip_atomic_load((const gu32_t *)(flag + idx),
                                                            __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT) == epoch;
            if (__all(ok)) break;
            if (spins >= BA_BACK_SPIN_MAX) {
                if (lane == 0) status[1] = 1.0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void cr32_publish(unsigned *flag, unsigned epoch, int nflags = 1)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
    __syncthreads();
    if (threadIdx.x < nflags)   // consecutive flag words (role 4: roles 0 and 1)
        __hip_atomic_store((gu32_t *)(flag + threadIdx.x), epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}


__global__ __launch_bounds__(256) void k_cr32_fused(double *S, long long lds, int TB, long long ld,
                                                    const int *__restrict__ elim,
                                                    const int *__restrict__ frec,
                                                    const int *__restrict__ srec, int nt,
                                                    double *linv, double *crL, double *rhs,
                                                    double *y, double *x, unsigned *flag,
                                                    unsigned long long *xg, unsigned epoch,
                                                    double *status, cr32_fplan P)
{
    CR32_LDS_DECL;
    CR_ST(0);
    const int b = blockIdx.x;
    int L = 0;
    while (L < P.nl && b >= P.b0[L + 1]) L++;
    // flag word of (level, tile, role): 3 = survivor's D_k, 4 = its r_k
    auto fw = [&](int lev, int t, int r) { return 5 * (lev * nt + t) + r; };
    if (L == 0) {
        // three records per tile, or two (roles 0 + 1 merged) when three would
        // not all fit on the CUs at once (one workgroup per CU)
        const int xr = P.l0two ? b / 2 : b / 3;
        const int role = P.l0two ? ((b & 1) ? 2 : 4) : b % 3;
        const int e = elim[3 * xr], p = elim[3 * xr + 1], q = elim[3 * xr + 2];
        CR_ST(1);
        if (!((role == 1 && p < 0) || (role == 2 && q < 0)))
            cr32_factor_body<true>(sh, S, lds, TB, ld, e, p, q, role, nt, linv, crL, rhs, y,
                                   status);
        CR_ST(2);
        if (role == 4)
            cr32_publish(flag + fw(0, e, 0), epoch, 2);
        else
            cr32_publish(flag + fw(0, e, role), epoch);
        CR_ST(3);
        return;
    }
    if (L < P.nl) {
        const int r = b - P.b0[L];
        const int ne = (P.b0[L + 1] - P.b0[L]) - (P.sofs[L + 1] - P.sofs[L]);   // 3 x fused
        int k, p = -1, q = -1, em, ep, role = 3;
        if (r >= ne) {
            const int *sr = srec + 3 * (P.sofs[L] + r - ne);
            k = sr[0];
            em = sr[1];
            ep = sr[2];
        } else {
            const int *fr = frec + 5 * (P.fofs[L] + r / 3);
            role = r % 3;
            k = fr[0];
            p = fr[1];
            q = fr[2];
            em = fr[3];
            ep = fr[4];
        }
        int w[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nw = 0;
        if (role == 1 || role == 2) {   // panels only: L(k, em), L(k, ep) and the fill's
            w[nw++] = fw(L - 1, em, 2);  // L(p, em) | L(q, ep) -- not role 0's y / L^-1
            if (role == 1) w[nw++] = fw(L - 1, em, 1);
            if (ep >= 0) {
                w[nw++] = fw(L - 1, ep, 1);
                if (role == 2) w[nw++] = fw(L - 1, ep, 2);
            }
            if (L >= 2) w[nw++] = fw(L - 1, k, 3);
        } else if (role == 3) {         // survivor, D_k first: L(k, em), L(k, ep)
            w[nw++] = fw(L - 1, em, 2);
            if (ep >= 0) w[nw++] = fw(L - 1, ep, 1);
            if (L >= 2) w[nw++] = fw(L - 1, k, 3);
        } else {
            for (int rr = 0; rr < 3; rr++) w[nw++] = fw(L - 1, em, rr);
            if (ep >= 0)
                for (int rr = 0; rr < 3; rr++) w[nw++] = fw(L - 1, ep, rr);
            if (L >= 2) {
                w[nw++] = fw(L - 1, k, 3);
                w[nw++] = fw(L - 1, k, 4);
            }
        }
        // (Tried in round 5: own D_k waited for alone and its loads issued
        // before the neighbours' wait -- 81 -> 86 us: the second poll-and-
        // barrier costs more than the overlapped loads save.)  BA_CR_PW: the
        // flags are polled per operand by the wave that loads it
        // (cr32_level_body), no poll-and-barrier here
        const bool skip = (role == 1 && p < 0) || (role == 2 && q < 0);
        if (!BA_CR_PW || skip) cr32_wait_flags(flag, nw, w, epoch, status);
        CR_ST(1);
        // the survivor's r_k: the neighbours' y and its own r_k of level L-1
        auto mid = [&]() {
            cr32_publish(flag + fw(L, k, 3), epoch);
            int w2[8] = {fw(L - 1, em, 0), 0, 0, 0, 0, 0, 0, 0}, n2 = 1;
            if (ep >= 0) w2[n2++] = fw(L - 1, ep, 0);
            if (L >= 2) w2[n2++] = fw(L - 1, k, 4);
            cr32_wait_flags(flag, n2, w2, epoch, status);
        };
        const cr32_pw pw{flag, epoch, status, L, nt};
        if (!skip)
            cr32_level_body<true>(sh, S, lds, TB, ld, k, p, q, em, ep, role, nt, linv, crL, rhs,
                                  y, status, mid, BA_CR_PW ? &pw : nullptr);
        CR_ST(2);
        cr32_publish(flag + fw(L, k, role == 3 ? 4 : role), epoch);
        CR_ST(3);
        return;
    }
    // back substitution, deepest record first
    const int rec = P.nrec - 1 - (b - P.b0[P.nl]);
    int Le = 0;
    while (Le + 1 < P.nl && rec >= P.eofs[Le + 1]) Le++;
    const int e = elim[3 * rec], p = elim[3 * rec + 1], q = elim[3 * rec + 2];
    const int w[8] = {fw(Le, e, 0), fw(Le, e, 1), fw(Le, e, 2), 0, 0, 0, 0, 0};
    cr32_wait_flags(flag, 3, w, epoch, status);
    CR_ST(1);
    cr32_back_body<true>(sh, e, p, q, nt, TB, ld, linv, crL, y, x, xg, epoch, status);
    CR_ST(2);
    CR_ST(3);
}

__global__ __launch_bounds__(256) void k_cr_back(const int *__restrict__ elim, int nt,
                                                 const double *__restrict__ linv,
                                                 const double *__restrict__ crL,
                                                 const double *__restrict__ y,
                                                 double *__restrict__ x)
{
    __shared__ double Ls[NB * LP];
    __shared__ double t[NB], u[NB];
    __shared__ double part[4][NB];
    const int tid = threadIdx.x;
    const int e = elim[3 * blockIdx.x], p = elim[3 * blockIdx.x + 1], q = elim[3 * blockIdx.x + 2];
    const long long T2 = (long long)NB * NB;
    if (tid < NB) t[tid] = y[(long long)NB * e + tid];
    if (p >= 0) {
        load_rowmajor(crL + T2 * e, Ls);
        if (tid < NB) u[tid] = x[(long long)NB * p + tid];
        __syncthreads();
        gemv64_t(Ls, u, part, u, 1.0);
        if (tid < NB) t[tid] -= u[tid];
        __syncthreads();
    }
    if (q >= 0) {
        load_rowmajor(crL + T2 * (nt + e), Ls);
        if (tid < NB) u[tid] = x[(long long)NB * q + tid];
        __syncthreads();
        gemv64_t(Ls, u, part, u, 1.0);
        if (tid < NB) t[tid] -= u[tid];
        __syncthreads();
    }
    load_rowmajor(linv + T2 * e, Ls);
    __syncthreads();
    gemv64_t(Ls, t, part, x + (long long)NB * e, 1.0);
}

// ---------------------------------------------------------------------------
// One launch builds every envelope tile of S for the factorisation: zeros
// (clearing the previous factorisation's in-place results and fill), the
// lower entries of the co-visible blocks that overlap the tile (S_jk, row >=
// col; bundle_euclid.m:192-193), and for diagonal tiles the pinv rule for
// exactly-zero rows (App. A Q2, Q8: unit diagonal, rhs 0; padding rows past
// NA*m included).  Workgroup 0 also clears the factorisation status.
// Replaces k_zero_env + k_assemble + k_fix_diag + two memsets (5 launches).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_assemble_tiles(
    double *__restrict__ S, long long lds, const int *__restrict__ env,
    const int *__restrict__ tb_ptr, const int *__restrict__ tb_blk,
    const int *__restrict__ blk_jk, const double *__restrict__ sblk, int na, long long ld,
    double *__restrict__ rhs, double *__restrict__ status, const int *__restrict__ crow,
    const int *__restrict__ rowsrc, const double *__restrict__ rhs_src)
{
    __shared__ double T[NB * (NB + 1)];
    const int ti = env[2 * blockIdx.x], tk = env[2 * blockIdx.x + 1], tid = threadIdx.x;
    for (int q = tid; q < NB * (NB + 1); q += 256) T[q] = 0.0;
    if (blockIdx.x == 0 && tid == 0) {
        status[0] = 0.0;   // non-positive pivot
        status[1] = 0.0;   // bounded hand-off spin gave up
    }
    __syncthreads();
    const long long r0 = (long long)NB * ti, c0 = (long long)NB * tk;
    const int na2 = na * na;
    const int u0 = tb_ptr[blockIdx.x], nq = (tb_ptr[blockIdx.x + 1] - u0) * na2;
    // (block, entry) pairs, all lanes busy; four a lane per step with their
    // three dependent loads (block id, its cameras, the entry) in flight
    // together -- each item writes its own tile entry, so the same tile
    for (int q0 = tid; q0 < nq; q0 += 4 * 256) {
        int lq[4], bq[4], jq[4], kq[4];
        double vq[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int q = min(q0 + 256 * t, nq - 1), u = q / na2;
            lq[t] = q - na2 * u;
            bq[t] = tb_blk[u0 + u];
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            jq[t] = blk_jk[2 * bq[t]];
            kq[t] = blk_jk[2 * bq[t] + 1];
            vq[t] = sblk[(size_t)na2 * bq[t] + lq[t]];
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
        if (q0 + 256 * t >= nq) break;
        const int l = lq[t], bj = jq[t], bc = kq[t];
        const int r = l % na, c = l / na;
        long long row, col;
        if (!crow) {
            row = (long long)na * bj + r;
            col = (long long)na * bc + c;
        } else {   // nested-dissection rows: S_kj = S_jk^T where camera k's rows come later
            row = crow[bj] + r;
            col = crow[bc] + c;
            if (row < col && bj != bc) {
                const long long t = row;
                row = col;
                col = t;
            }
        }
        if (row < col || row < r0 || row >= r0 + NB || col < c0 || col >= c0 + NB) continue;
        T[(row - r0) * (NB + 1) + (col - c0)] = vq[t];
        }
    }
    __syncthreads();
    if (ti == tk && tid < NB) {   // pinv semantics for exactly-zero rows, padding rows
        double *d = T + tid * (NB + 1) + tid;
        const long long r = r0 + tid;
        if (rowsrc) {   // gather the row-ordered rhs (nested dissection)
            const int src = rowsrc[r];
            rhs[r] = src >= 0 ? rhs_src[src] : 0.0;
        }
        if (*d == 0.0) {
            *d = 1.0;
            rhs[r] = 0.0;
        } else if (r >= ld) {
            rhs[r] = 0.0;
        }
    }
    __syncthreads();
    double *base = S + r0 + lds * c0;
    const int r = tid & 63, cq = tid >> 6;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int c = cq + 4 * u;
        base[r + lds * c] = T[r * (NB + 1) + c];
    }
}

// zero every envelope tile of S (fill from the previous factorisation)
__global__ void k_zero_env(double *__restrict__ S, long long lds, const int *__restrict__ env)
{
    const int i = env[2 * blockIdx.x], k = env[2 * blockIdx.x + 1];
    double *base = S + (long long)NB * i + lds * (long long)NB * k;
    for (int q = threadIdx.x; q < NB * NB; q += blockDim.x) {
        const int r = q & (NB - 1), c = q >> 6;
        base[r + lds * c] = 0.0;
    }
}

// pinv semantics for exactly-zero rows (App. A Q2, Q8): such a row/column of
// S is exactly zero (its A columns are zero, hence its W and Y rows); give it
// a unit diagonal and a zero right-hand side so da = 0 there.
__global__ void k_fix_diag(double *__restrict__ S, double *__restrict__ rhs, long long lds)
{
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= lds) return;
    double *d = S + r + lds * r;
    if (*d == 0.0) {
        *d = 1.0;
        rhs[r] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// Sequential reduced solve (dense_solve = 3, the parity mode): left-looking
// Cholesky of the lower triangle, every sum in ascending index order, then the
// two triangular solves -- exactly the loops of the CPU oracle's
// sequential Cholesky, so da is bit-identical to it.  One
// workgroup: the diagonal entry of column j by lane 0, the column's rows by
// the other lanes (each row's sum stays sequential).  The exactly-zero rows
// have their unit diagonal / zero rhs from k_assemble_tiles (App. A Q8).
// For the small problems of the parity tests (ld of a few hundred).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_seq(double *__restrict__ S, long long lds,
                                                  int n, double *__restrict__ rhs,
                                                  double *__restrict__ x,
                                                  double *__restrict__ status)
{
    __shared__ double piv;
    __shared__ int bad;
    const int tid = threadIdx.x;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int j = 0; j < n; j++) {
        if (tid == 0) {
            double s = S[j + lds * j];
            for (int k = 0; k < j; k++) {
                const double l = S[j + lds * k];
                s = s - l * l;
            }
            if (!(s > 0.0)) bad = 1;
            piv = sqrt(s);
            S[j + lds * j] = piv;
        }
        __syncthreads();
        if (bad) break;
        const double p = piv;
        for (int i = j + 1 + tid; i < n; i += 256) {
            double t = S[i + lds * j];
            for (int k = 0; k < j; k++) t = t - S[i + lds * k] * S[j + lds * k];
            S[i + lds * j] = t / p;
        }
        __syncthreads();
    }
    if (bad) {
        if (tid == 0) status[0] = 1.0;
        return;
    }
    if (tid == 0) {   // L y = rhs, then L^T x = y (x over y in place)
        for (int i = 0; i < n; i++) {
            double t = rhs[i];
            for (int k = 0; k < i; k++) t = t - S[i + lds * k] * x[k];
            x[i] = t / S[i + lds * i];
        }
        for (int i = n - 1; i >= 0; i--) {
            double t = x[i];
            for (int k = i + 1; k < n; k++) t = t - S[k + lds * i] * x[k];
            x[i] = t / S[i + lds * i];
        }
    }
}

// ---------------------------------------------------------------------------
// pinv(S) e_ from the symmetric eigen-decomposition (the fallback when the
// Cholesky meets a non-positive pivot: bundle_euclid.m:193 always takes
// pinv(S)*e_).  MATLAB's pinv keeps the singular values
// (= |eigenvalues| here) above max(size) * eps(max singular value).
//   k_pinv_w: w_k = (v_k . rhs) / ev_k  for |ev_k| > tol, else 0
//   k_pinv_x: da_i = sum_k V[i][k] w_k
// one workgroup per output entry, fixed-order reductions (deterministic).
// ---------------------------------------------------------------------------
static __device__ double dev_eps_of(double x)
{
    if (!(x > 0.0)) return 4.9406564584124654e-324;
    int e;
    (void)frexp(x, &e);
    return ldexp(1.0, e - 53);
}

__global__ __launch_bounds__(256) void k_pinv_w(const double *__restrict__ V,
                                                const double *__restrict__ ev, long long ld,
                                                const double *__restrict__ rhs,
                                                double *__restrict__ w)
{
    __shared__ double red[256];
    const long long k = blockIdx.x;
    double acc = 0.0;
    for (long long i = threadIdx.x; i < ld; i += 256) acc += V[i + ld * k] * rhs[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double emax = fmax(fabs(ev[0]), fabs(ev[ld - 1]));
        const double tol = (double)ld * dev_eps_of(emax);
        w[k] = fabs(ev[k]) > tol ? red[0] / ev[k] : 0.0;
    }
}

__global__ __launch_bounds__(256) void k_pinv_x(const double *__restrict__ V, long long ld,
                                                const double *__restrict__ w,
                                                double *__restrict__ da)
{
    __shared__ double red[256];
    const long long i = blockIdx.x;
    double acc = 0.0;
    for (long long k = threadIdx.x; k < ld; k += 256) acc += V[i + ld * k] * w[k];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) da[i] = red[0];
}

int ba_pinv_apply(ba_dev *d, const double *V, const double *ev, long long ld, const double *rhs,
                  double *work, double *da)
{
    if (ld <= 0) return 0;
    k_pinv_w<<<(unsigned)ld, 256, 0, d->stream>>>(V, ev, ld, rhs, work);
    k_pinv_x<<<(unsigned)ld, 256, 0, d->stream>>>(V, ld, work, da);
    return -(int)hipGetLastError();
}

// ===========================================================================
template <typename T>
static int dev_alloc(T **p, size_t bytes)
{
    *p = (T *)ba_dmalloc(bytes);
    return *p ? 0 : -(int)hipErrorOutOfMemory;
}

// ---- nested dissection of the envelope (host planner) -------------------
namespace {
struct nd_cost_t {
    int crit, ns, n[BA_ND_MAX];
};

// arcs [bnd[t], bnd[t+1]) of consecutive cameras; camera j of arc t joins the
// separator when it is co-visible with a camera of an earlier arc (minK[j] <
// bnd[t]).  Predicted step chain: the longest arc, the separator's columns,
// and the two SYRK launches between them.
nd_cost_t nd_cost(const std::vector<int> &minK, int na, const int *bnd, int K)
{
    nd_cost_t e{};
    int nsep = 0, mx = 0;
    for (int t = 0; t < K; t++) {
        int cnt = 0;
        for (int j = bnd[t]; j < bnd[t + 1]; j++) {
            if (minK[j] < bnd[t])
                nsep++;
            else
                cnt++;
        }
        e.n[t] = (na * cnt + NB - 1) / NB;
        mx = std::max(mx, e.n[t]);
    }
    e.ns = (na * nsep + NB - 1) / NB;
    e.crit = mx + e.ns + (e.ns > 0 ? 2 : 0);
    return e;
}

// K = 2 .. BA_ND_MAX arcs: equal camera counts, then one boundary at a time
// moved while the predicted chain shortens.  Returns the best K (0: none).
int nd_choose(const std::vector<int> &minK, int m, int na, int *bnd_out, int &crit_out)
{
    int bestK = 0;
    crit_out = INT_MAX;
    for (int K = 2; K <= BA_ND_MAX && K <= m; K++) {
        int bnd[BA_ND_MAX + 1];
        for (int t = 0; t <= K; t++) bnd[t] = (int)((long long)t * m / K);
        nd_cost_t cur = nd_cost(minK, na, bnd, K);
        for (int sweep = 0; sweep < 4; sweep++) {
            bool moved = false;
            for (int t = 1; t < K; t++)
                for (int step = std::max(1, m / (4 * K)); step >= 1; step /= 2)
                    for (int dir = -1; dir <= 1; dir += 2)
                        for (;;) {
                            const int nbd = bnd[t] + dir * step;
                            if (nbd <= bnd[t - 1] || nbd >= bnd[t + 1]) break;
                            const int keep = bnd[t];
                            bnd[t] = nbd;
                            const nd_cost_t c = nd_cost(minK, na, bnd, K);
                            if (c.crit < cur.crit) {
                                cur = c;
                                moved = true;
                            } else {
                                bnd[t] = keep;
                                break;
                            }
                        }
            if (!moved) break;
        }
        if (cur.crit < crit_out) {
            crit_out = cur.crit;
            bestK = K;
            for (int t = 0; t <= K; t++) bnd_out[t] = bnd[t];
        }
    }
    return bestK;
}
}   // namespace

static std::vector<int> nd_min_cam(int m, const int *blk_jk, int nb)
{
    std::vector<int> minK(m);
    for (int j = 0; j < m; j++) minK[j] = j;
    for (int b = 0; b < nb; b++) {
        const int j = blk_jk[2 * b], k = blk_jk[2 * b + 1];
        if (k < minK[j]) minK[j] = k;
    }
    return minK;
}

extern "C" int vlgba_debug_nd_plan(int m, int num_a, const int *blk_jk, int nb, int *bnd,
                                   int *crit)
{
    if (m < 2 || num_a < 1 || nb < 0 || (nb > 0 && !blk_jk) || !bnd || !crit) return -1;
    for (int b = 0; b < nb; b++)
        if (blk_jk[2 * b] < blk_jk[2 * b + 1] || blk_jk[2 * b + 1] < 0 || blk_jk[2 * b] >= m)
            return -1;
    return nd_choose(nd_min_cam(m, blk_jk, nb), m, num_a, bnd, *crit);
}

int ba_chol_setup(ba_dev *d, const int *blk_jk, int nb)
{
    int nt = (int)(d->lds / NB);
    d->nt = nt;
    d->h_tfirst = new int[nt];
    d->fl_factor = d->fl_syrk = d->fl_back = 0.0;
    // every lower tile for the measurement mode (1) and the sequential parity
    // solve (3); the envelope otherwise (0 auto, 2 envelope without CR, 4 ND)
    const bool all_tiles = d->dense_solve == 1 || d->dense_solve == 3;
    for (int i = 0; i < nt; i++) d->h_tfirst[i] = all_tiles ? 0 : i;
    if (!all_tiles)
        for (int b = 0; b < nb; b++) {
            const int j = blk_jk[2 * b], k = blk_jk[2 * b + 1];   // j >= k
            const long long r0 = (long long)d->na * j, c0 = (long long)d->na * k;
            for (long long r = r0; r < r0 + d->na; r++) {
                const int ti = (int)(r / NB);
                const int tk = (int)(c0 / NB);
                if (tk < d->h_tfirst[ti]) d->h_tfirst[ti] = tk;
            }
        }
    // cyclic reduction when S is tile-tridiagonal (dense_solve 0 = auto):
    // camera-aligned 32-row tiles when the co-visibility band allows them
    // (every block (j, k) within neighbouring groups of floor(32 / NA)
    // cameras), else the 64-row tiles
    d->cr_nlev = 0;
    d->cr32 = 0;
    int ntc = nt;
    if (d->dense_solve == 0 && d->na <= 32) {
        const int G = 32 / d->na, TB = d->na * G;
        const int nt32 = (int)((d->ld + TB - 1) / TB);
        bool ok = nt32 > 1;
        for (int b = 0; ok && b < nb; b++) {
            const int dj = blk_jk[2 * b] / G - blk_jk[2 * b + 1] / G;
            if (dj > 1 || dj < -1) ok = false;
        }
        if (ok) {
            d->cr32 = 1;
            d->tb32 = TB;
            d->nt32 = nt32;
            ntc = nt32;
            // direct assembly: every camera pair (j >= k) inside a group of G
            // cameras is a block (the diagonal tiles the CR writes back are then
            // fully rewritten by k_schur_reduce every pass)
            long long inside = 0, want = 0;
            for (int b = 0; b < nb; b++)
                inside += blk_jk[2 * b] / G == blk_jk[2 * b + 1] / G;
            for (int g0 = 0; g0 < d->m; g0 += G) {
                const long long c = std::min(G, d->m - g0);
                want += c * (c + 1) / 2;
            }
            d->asm_direct_ok = inside == want;
        }
    }
    bool tridiag = d->dense_solve == 0 && nt > 1;
    for (int i = 1; tridiag && i < nt; i++)
        if (d->h_tfirst[i] < i - 1) tridiag = false;
    if (d->cr32) tridiag = true;
    if (tridiag) {
        const int nt = ntc;   // the CR tile count (64- or camera-aligned 32-row tiles)
        std::vector<int> act(nt), elim, keep, eptr{0}, kptr{0};
        for (int i = 0; i < nt; i++) act[i] = i;
        while (!act.empty()) {
            const int len = (int)act.size();
            std::vector<int> next;
            for (int t = 0; t < len; t++) {
                if ((t & 1) == 0) {
                    elim.push_back(act[t]);
                    elim.push_back(t > 0 ? act[t - 1] : -1);
                    elim.push_back(t + 1 < len ? act[t + 1] : -1);
                } else {
                    keep.push_back(act[t]);
                    keep.push_back(act[t - 1]);
                    keep.push_back(t + 1 < len ? act[t + 1] : -1);
                    keep.push_back(t + 2 < len ? act[t + 2] : -1);
                    next.push_back(act[t]);
                }
            }
            eptr.push_back((int)elim.size() / 3);
            kptr.push_back((int)keep.size() / 4);
            act.swap(next);
        }
        d->cr_nlev = (int)eptr.size() - 1;
        {   // the CR's algorithmic flops (ba_dev::fl_factor): per elimination
            // record (e, p, q) the factor + inverse of D_e, y_e and one panel per
            // neighbour; per kept record (k, e-, e+, k2) the update of D_k and r_k
            // by its eliminated neighbours and the fill towards k2; the back
            // substitution's GEMVs
            const double t = d->cr32 ? T32 : NB;
            const double potri = 2.0 * t * t * t / 3.0, gemm = 2.0 * t * t * t, gemv = 2.0 * t * t;
            d->fl_factor = d->fl_syrk = d->fl_back = 0.0;
            for (size_t i = 0; i < elim.size(); i += 3) {
                const double nbr = (elim[i + 1] >= 0) + (elim[i + 2] >= 0);
                d->fl_factor += potri + gemv + nbr * gemm;
                d->fl_back += (nbr + 1) * gemv;
            }
            for (size_t i = 0; i < keep.size(); i += 4) {
                const double nbe = 1 + (keep[i + 2] >= 0);
                d->fl_factor += nbe * (gemm + gemv) + (keep[i + 3] >= 0) * gemm;
            }
        }
        if (d->cr32) {   // the fused levels' records (see k_cr32_level)
            const int nl = d->cr_nlev;
            std::vector<int> frec, srec, fptr(nl + 1, 0), sptr(nl + 1, 0);
            std::vector<int> em_of(nt, -1), ep_of(nt, -1);
            for (int L = 1; L < nl; L++) {
                for (int i = kptr[L - 1]; i < kptr[L]; i++) {
                    em_of[keep[4 * i]] = keep[4 * i + 1];
                    ep_of[keep[4 * i]] = keep[4 * i + 2];
                }
                for (int i = eptr[L]; i < eptr[L + 1]; i++) {
                    const int e = elim[3 * i];
                    frec.insert(frec.end(), {e, elim[3 * i + 1], elim[3 * i + 2], em_of[e],
                                             ep_of[e]});
                }
                for (int i = kptr[L]; i < kptr[L + 1]; i++) {
                    const int k = keep[4 * i];
                    srec.insert(srec.end(), {k, em_of[k], ep_of[k]});
                }
                fptr[L + 1] = (int)frec.size() / 5;
                sptr[L + 1] = (int)srec.size() / 3;
            }
            fptr[1] = 0;
            sptr[1] = 0;
            d->crf_ptr_h = new int[nl + 1];
            d->crs_ptr_h = new int[nl + 1];
            for (int L = 0; L <= nl; L++) {
                d->crf_ptr_h[L] = L >= 1 ? fptr[L] : 0;
                d->crs_ptr_h[L] = L >= 1 ? sptr[L] : 0;
            }
            TRY_RC(dev_alloc(&d->xgran, sizeof(unsigned long long) * 64 * (size_t)nt));
            VLGBA_CHECK(hipMemsetAsync(d->xgran, 0, sizeof(unsigned long long) * 64 * (size_t)nt,
                                       d->stream));
            d->back_epoch = 0;
            {   // one-launch CR (k_cr32_fused) unless VLGBA_CR_FUSED=0
                const char *ev = std::getenv("VLGBA_CR_FUSED");
                d->cr_fused = !(ev && ev[0] == '0') && nl <= BA_CR_MAXLEV;
            }
            if (d->cr_fused) {
                const size_t nfl = (size_t)5 * nl * nt;
                TRY_RC(dev_alloc(&d->crflag, sizeof(unsigned) * nfl));
                VLGBA_CHECK(hipMemsetAsync(d->crflag, 0, sizeof(unsigned) * nfl, d->stream));
            }
            TRY_RC(dev_alloc(&d->crf, sizeof(int) * (frec.size() + 1)));
            TRY_RC(dev_alloc(&d->crs, sizeof(int) * (srec.size() + 1)));
            if (!frec.empty())
                VLGBA_CHECK(hipMemcpyAsync(d->crf, frec.data(), sizeof(int) * frec.size(),
                                           hipMemcpyHostToDevice, d->stream));
            if (!srec.empty())
                VLGBA_CHECK(hipMemcpyAsync(d->crs, srec.data(), sizeof(int) * srec.size(),
                                           hipMemcpyHostToDevice, d->stream));
            VLGBA_CHECK(hipStreamSynchronize(d->stream));
        }
        d->cr_eptr_h = new int[eptr.size()];
        d->cr_kptr_h = new int[kptr.size()];
        for (size_t q = 0; q < eptr.size(); q++) d->cr_eptr_h[q] = eptr[q];
        for (size_t q = 0; q < kptr.size(); q++) d->cr_kptr_h[q] = kptr[q];
        TRY_RC(dev_alloc(&d->cr_elim, sizeof(int) * elim.size()));
        TRY_RC(dev_alloc(&d->cr_keep, sizeof(int) * (keep.size() + 1)));
        TRY_RC(dev_alloc(&d->crL, sizeof(double) * 2 * (size_t)nt *
                                      (d->cr32 ? T32 * T32 : NB * NB)));
        VLGBA_CHECK(hipMemcpyAsync(d->cr_elim, elim.data(), sizeof(int) * elim.size(),
                                   hipMemcpyHostToDevice, d->stream));
        if (!keep.empty())
            VLGBA_CHECK(hipMemcpyAsync(d->cr_keep, keep.data(), sizeof(int) * keep.size(),
                                       hipMemcpyHostToDevice, d->stream));
    }
    // nested dissection (not for tridiagonal S, which the cyclic reduction takes)
    d->nd_np = 0;
    {
        const char *eg = std::getenv("VLGBA_ND_GROUPED");
        d->nd_grouped = !(eg && eg[0] == '0');
    }
    const int na = d->na, m = d->m;
    std::vector<int> crow, tpart;   // row of camera j; part of tile (arc t, separator np)
    if (!tridiag && (d->dense_solve == 0 || d->dense_solve == 4) && m >= 2 && nt > 1) {
        const char *ev = std::getenv("VLGBA_ND");
        const bool off = ev && ev[0] == '0';
        const std::vector<int> minK = nd_min_cam(m, blk_jk, nb);
        int bnd[BA_ND_MAX + 1], crit = INT_MAX;
        const int K = off && d->dense_solve == 0 ? 0 : nd_choose(minK, m, na, bnd, crit);
        bool take = K > 0 && (d->dense_solve == 4 || (nt >= 8 && 4 * crit <= 3 * nt));
        // setup budget: the separator SYRK's host lists cost
        // O(ns^2 s0) and its partials (pairs + CUs) x 33 KB of device memory --
        // a graph with a wide separator keeps the natural order instead
        long long npair_max = 0, setup_ops = 0;
        if (K > 0) {
            const nd_cost_t c = nd_cost(minK, na, bnd, K);
            long long s0t = 0;
            for (int t = 0; t < K; t++) s0t += c.n[t];
            npair_max = (long long)c.ns * (c.ns + 1) / 2;
            setup_ops = npair_max * s0t;
            if (npair_max > BA_ND_MAX_PAIRS || setup_ops > BA_ND_MAX_SETUP) take = false;
        }
        if (ev && ev[0] == 'v')
            std::fprintf(stderr, "[vlgba] nested dissection: natural %d tiles, %d arcs -> chain %d, "
                         "<= %lld separator pairs, %lld setup checks%s\n", nt, K, crit, npair_max,
                         setup_ops, take ? "" : " (not taken)");
        if (take) {
            crow.assign(m, -1);
            long long row = 0;
            for (int t = 0; t < K; t++) {
                d->nd_a0[t] = (int)(row / NB);
                for (int j = bnd[t]; j < bnd[t + 1]; j++)
                    if (minK[j] >= bnd[t]) {
                        crow[j] = (int)row;
                        row += na;
                    }
                row = (row + NB - 1) / NB * NB;
            }
            d->nd_a0[K] = (int)(row / NB);
            for (int t = 0; t < K; t++)
                for (int j = bnd[t]; j < bnd[t + 1]; j++)
                    if (minK[j] < bnd[t]) {
                        crow[j] = (int)row;
                        row += na;
                    }
            row = (row + NB - 1) / NB * NB;
            d->nd_np = K;
            d->slds = row;
            nt = (int)(row / NB);
            d->nt = nt;
            tpart.assign(nt, K);
            for (int t = 0; t < K; t++)
                for (int i = d->nd_a0[t]; i < d->nd_a0[t + 1]; i++) tpart[i] = t;
        }
    }
    const bool nd = d->nd_np > 0;
    const int npart = nd ? d->nd_np + 1 : 1;
    const int s0 = nd ? d->nd_a0[d->nd_np] : nt;
    // first[i][P]: the first envelope tile of row i among the columns of part P
    // (the profile is preserved inside each part: arcs never couple, and the
    // separator block fills in, so it is taken dense)
    std::vector<int> first;
    if (nd) {
        delete[] d->h_tfirst;
        d->h_tfirst = new int[nt];
        first.assign((size_t)nt * npart, INT_MAX);
        for (int i = 0; i < nt; i++) first[(size_t)i * npart + tpart[i]] = i >= s0 ? s0 : i;
        for (int b = 0; b < nb; b++) {
            long long r0 = crow[blk_jk[2 * b]], c0 = crow[blk_jk[2 * b + 1]];
            if (r0 < c0) std::swap(r0, c0);
            const int tk = (int)(c0 / NB), P = tpart[tk];
            for (long long r = r0; r < r0 + na; r++) {
                int &f = first[(size_t)(r / NB) * npart + P];
                if (tk < f) f = tk;
            }
        }
        for (int i = 0; i < nt; i++) {
            int f = i;
            for (int P = 0; P < npart; P++) f = std::min(f, first[(size_t)i * npart + P]);
            d->h_tfirst[i] = f;
        }
    } else {
        first.assign(d->h_tfirst, d->h_tfirst + nt);
    }
    auto in_env = [&](int i, int k) { return first[(size_t)i * npart + (nd ? tpart[k] : 0)] <= k; };
    std::vector<int> ptr(nt + 1, 0), list, env;
    for (int k = 0; k < nt; k++) {
        for (int i = k + 1; i < nt; i++)
            if (in_env(i, k)) list.push_back(i);
        ptr[k + 1] = (int)list.size();
    }
    for (int k = 0; k < nt; k++)
        for (int i = k; i < nt; i++)
            if (in_env(i, k)) {
                env.push_back(i);
                env.push_back(k);
            }
    d->n_env = (int)env.size() / 2;
    {   // per envelope tile: the co-visible blocks (j >= k) overlapping it
        std::vector<int> tid_of((size_t)nt * nt, -1);
        for (int e = 0; e < d->n_env; e++) tid_of[(size_t)env[2 * e] * nt + env[2 * e + 1]] = e;
        std::vector<std::vector<int>> lists(d->n_env);
        for (int b = 0; b < nb; b++) {
            long long r0 = (long long)na * blk_jk[2 * b], c0 = (long long)na * blk_jk[2 * b + 1];
            if (nd) {
                r0 = crow[blk_jk[2 * b]];
                c0 = crow[blk_jk[2 * b + 1]];
                if (r0 < c0) std::swap(r0, c0);
            }
            const int t0 = (int)(r0 / NB), t1 = (int)((r0 + na - 1) / NB);
            const int u0 = (int)(c0 / NB), u1 = (int)((c0 + na - 1) / NB);
            for (int t = t0; t <= t1; t++)
                for (int u = u0; u <= u1 && u <= t; u++) {
                    const int e = tid_of[(size_t)t * nt + u];
                    if (e >= 0) lists[e].push_back(b);
                }
        }
        std::vector<int> tptr(d->n_env + 1, 0), tblk;
        for (int e = 0; e < d->n_env; e++) {
            tblk.insert(tblk.end(), lists[e].begin(), lists[e].end());
            tptr[e + 1] = (int)tblk.size();
        }
        TRY_RC(dev_alloc(&d->tb_ptr, sizeof(int) * tptr.size()));
        TRY_RC(dev_alloc(&d->tb_blk, sizeof(int) * (tblk.size() + 1)));
        VLGBA_CHECK(hipMemcpyAsync(d->tb_ptr, tptr.data(), sizeof(int) * tptr.size(),
                                   hipMemcpyHostToDevice, d->stream));
        if (!tblk.empty())
            VLGBA_CHECK(hipMemcpyAsync(d->tb_blk, tblk.data(), sizeof(int) * tblk.size(),
                                       hipMemcpyHostToDevice, d->stream));
        VLGBA_CHECK(hipStreamSynchronize(d->stream));
    }
    // the factor's storage: S (dense, column major), the diagonal tiles'
    // inverses, the forward-solve result (+ the 32-row CR's last tile)
    const long long sdim = nd ? d->slds : d->lds;
    TRY_RC(dev_alloc(&d->S, sizeof(double) * (size_t)(sdim * sdim)));
    TRY_RC(dev_alloc(&d->linv, sizeof(double) * (size_t)(sdim / NB) * NB * NB));
    TRY_RC(dev_alloc(&d->ywork, sizeof(double) * (size_t)(sdim + NB)));
    if (nd) {
        std::vector<int> rowsrc(d->slds, -1), prow(d->lds, -1);
        for (int j = 0; j < m; j++)
            for (int r = 0; r < na; r++) {
                rowsrc[crow[j] + r] = na * j + r;
                prow[(size_t)na * j + r] = crow[j] + r;
            }
        // separator pairs (i >= j, ascending) and their arc columns, chunked
        std::vector<int> pairs, pptr{0}, rec, klist;
        std::vector<std::vector<int>> kl;
        long long work = 0;
        for (int i = s0; i < nt; i++)
            for (int j = s0; j <= i; j++) {
                std::vector<int> ks;
                for (int k = 0; k < s0; k++)
                    if (in_env(i, k) && in_env(j, k)) ks.push_back(k);
                if (ks.empty()) continue;
                work += (long long)ks.size();
                pairs.push_back(i);
                pairs.push_back(j);
                kl.push_back(std::move(ks));
            }
        const int kc = (int)std::max<long long>(2, (work + d->ncu - 1) / std::max(1, d->ncu));
        for (size_t p = 0; p < kl.size(); p++) {
            for (size_t q = 0; q < kl[p].size(); q += kc) {
                rec.push_back((int)p);
                rec.push_back((int)klist.size());
                const int cnt = (int)std::min<size_t>(kc, kl[p].size() - q);
                rec.push_back(cnt);
                klist.insert(klist.end(), kl[p].begin() + q, kl[p].begin() + q + cnt);
            }
            pptr.push_back((int)rec.size() / 3);
        }
        d->fl_syrk = (double)work * 2.0 * NB * NB * NB +
                     (double)(pairs.size() / 2) * 2.0 * NB * NB;
        d->nd_npair = (int)pairs.size() / 2;
        d->nd_nrec = (int)rec.size() / 3;
        auto up = [&](int **dst, const std::vector<int> &v) -> int {
            TRY_RC(dev_alloc(dst, sizeof(int) * (v.size() + 1)));
            if (!v.empty())
                VLGBA_CHECK(hipMemcpyAsync(*dst, v.data(), sizeof(int) * v.size(),
                                           hipMemcpyHostToDevice, d->stream));
            return 0;
        };
        TRY_RC(up(&d->nd_crow, crow));
        TRY_RC(up(&d->nd_prow, prow));
        TRY_RC(up(&d->nd_rowsrc, rowsrc));
        TRY_RC(up(&d->nd_pair, pairs));
        TRY_RC(up(&d->nd_pptr, pptr));
        TRY_RC(up(&d->nd_rec, rec));
        TRY_RC(up(&d->nd_klist, klist));
        TRY_RC(dev_alloc(&d->nd_rhs, sizeof(double) * (size_t)d->slds));
        TRY_RC(dev_alloc(&d->nd_x, sizeof(double) * (size_t)d->slds));
        TRY_RC(dev_alloc(&d->nd_part, sizeof(double) * ((size_t)d->nd_nrec + 1) * (NB * NB + NB)));
        VLGBA_CHECK(hipStreamSynchronize(d->stream));
    }
    {   // the envelope's algorithmic flops (see ba_dev::fl_factor; the CR's: above)
        const double t = NB;
        const double potri = 2.0 * t * t * t / 3.0, gemm = 2.0 * t * t * t, gemv = 2.0 * t * t;
        for (int k = 0; k < nt && !d->cr_nlev && d->dense_solve != 3; k++) {
            const double T = ptr[k + 1] - ptr[k];
            // factor + inverse, y_k, T panels and their rhs updates, the trailing
            // pairs of column k (applied in step k + 1; an arc column's separator
            // x separator pairs go to the separator SYRK instead)
            double nsr = 0;
            if (nd && k < s0)
                for (int q = ptr[k]; q < ptr[k + 1]; q++) nsr += list[q] >= s0;
            d->fl_factor += potri + gemv + T * (gemm + gemv) +
                            (T * (T + 1) / 2 - nsr * (nsr + 1) / 2) * gemm;
            d->fl_back += (T + 1) * gemv;
        }
        if (d->cr_nlev > 0 && d->cr_fused) {   // one CR launch: timed as k_cr_factor
            d->fl_factor += d->fl_back;
            d->fl_back = 0.0;
        }
    }
    d->pan_ptr_h = new int[nt + 1];
    for (int k = 0; k <= nt; k++) d->pan_ptr_h[k] = ptr[k];
    d->h_pan_list = new int[list.size() + 1];
    for (size_t q = 0; q < list.size(); q++) d->h_pan_list[q] = list[q];
    TRY_RC(dev_alloc(&d->pan_list, sizeof(int) * (list.size() + 1)));
    if (!d->cr_nlev && d->dense_solve != 3 && nt <= d->ncu) {   // one-launch backward
        TRY_RC(dev_alloc(&d->pan_ptr, sizeof(int) * (nt + 1)));
        VLGBA_CHECK(hipMemcpyAsync(d->pan_ptr, ptr.data(), sizeof(int) * (nt + 1),
                                   hipMemcpyHostToDevice, d->stream));
        TRY_RC(dev_alloc(&d->xgran64, sizeof(unsigned long long) * 128 * (size_t)nt));
        VLGBA_CHECK(hipMemsetAsync(d->xgran64, 0, sizeof(unsigned long long) * 128 * (size_t)nt,
                                   d->stream));
        d->back_epoch = 0;
    }
    if (!d->cr_nlev && d->dense_solve != 3) {   // the factor's in-launch hand-off
        TRY_RC(dev_alloc(&d->kflag, sizeof(unsigned) * (size_t)nt));
        VLGBA_CHECK(hipMemsetAsync(d->kflag, 0, sizeof(unsigned) * (size_t)nt, d->stream));
        d->fac_epoch = 0;
        // runner mode's flags: lflag | dflag | uflag | pflag, nt each, then
        // the runner's timeout word.  Opt-in (VLGBA_ENV_RUNNER=1): the runner
        // makes progress only while its stream has a hardware queue of its own
        const char *er = std::getenv("VLGBA_ENV_RUNNER");
        d->env_runner = er && er[0] == '1';
        if (d->env_runner && d->pan_ptr) {
            const size_t nw = 4 * (size_t)nt + 1;
            TRY_RC(dev_alloc(&d->rflag, sizeof(unsigned) * nw));
            VLGBA_CHECK(hipMemsetAsync(d->rflag, 0, sizeof(unsigned) * nw, d->stream));
        }
    }
    TRY_RC(dev_alloc(&d->env_tiles, sizeof(int) * (env.size() + 1)));
    if (!list.empty())
        VLGBA_CHECK(hipMemcpyAsync(d->pan_list, list.data(), sizeof(int) * list.size(),
                                   hipMemcpyHostToDevice, d->stream));
    VLGBA_CHECK(hipMemcpyAsync(d->env_tiles, env.data(), sizeof(int) * env.size(),
                               hipMemcpyHostToDevice, d->stream));
    VLGBA_CHECK(hipMemsetAsync(d->S, 0, sizeof(double) * sdim * sdim, d->stream));
    VLGBA_CHECK(hipStreamSynchronize(d->stream));
    return 0;
}

void ba_chol_free(ba_dev *d)
{
    for (void *q : {(void *)d->S, (void *)d->linv, (void *)d->ywork, (void *)d->nd_crow,
                    (void *)d->nd_prow, (void *)d->nd_rowsrc, (void *)d->nd_rhs, (void *)d->nd_x,
                    (void *)d->nd_pair, (void *)d->nd_pptr, (void *)d->nd_rec, (void *)d->nd_klist,
                    (void *)d->nd_part})
        if (q) ba_dfree(q);
    d->S = d->linv = d->ywork = d->nd_rhs = d->nd_x = d->nd_part = nullptr;
    d->nd_crow = d->nd_prow = d->nd_rowsrc = d->nd_pair = d->nd_pptr = d->nd_rec = d->nd_klist =
        nullptr;
    d->nd_np = 0;
    delete[] d->h_tfirst;
    delete[] d->pan_ptr_h;
    delete[] d->h_pan_list;
    d->h_pan_list = nullptr;
    delete[] d->cr_eptr_h;
    delete[] d->cr_kptr_h;
    d->cr_eptr_h = d->cr_kptr_h = nullptr;
    if (d->xgran) ba_dfree(d->xgran);
    d->xgran = nullptr;
    if (d->rflag) ba_dfree(d->rflag);
    d->rflag = nullptr;
    d->rstream = nullptr;   // the process's (env_runner_stream)
    if (d->crflag) ba_dfree(d->crflag);
    d->crflag = nullptr;
    d->cr_fused = 0;
    if (d->crf) ba_dfree(d->crf);
    if (d->crs) ba_dfree(d->crs);
    delete[] d->crf_ptr_h;
    delete[] d->crs_ptr_h;
    d->crf = d->crs = nullptr;
    d->crf_ptr_h = d->crs_ptr_h = nullptr;
    if (d->cr_elim) ba_dfree(d->cr_elim);
    if (d->cr_keep) ba_dfree(d->cr_keep);
    if (d->crL) ba_dfree(d->crL);
    d->cr_elim = d->cr_keep = nullptr;
    d->crL = nullptr;
    d->cr_nlev = 0;
    if (d->tb_ptr) ba_dfree(d->tb_ptr);
    if (d->tb_blk) ba_dfree(d->tb_blk);
    d->tb_ptr = d->tb_blk = nullptr;
    if (d->pan_list) ba_dfree(d->pan_list);
    if (d->pan_ptr) ba_dfree(d->pan_ptr);
    if (d->xgran64) ba_dfree(d->xgran64);
    if (d->kflag) ba_dfree(d->kflag);
    d->pan_ptr = nullptr;
    d->xgran64 = nullptr;
    d->kflag = nullptr;
    if (d->env_tiles) ba_dfree(d->env_tiles);
    d->h_tfirst = d->pan_ptr_h = nullptr;
    d->pan_list = d->env_tiles = nullptr;
}

int ba_assemble_tiles(ba_dev *d)
{
    if (d->asm_direct) return 0;   // k_schur_reduce wrote S (and reset the status)
    const bool nd = d->nd_np > 0;
    k_assemble_tiles<<<d->n_env, 256, 0, d->stream>>>(
        d->S, nd ? d->slds : d->lds, d->env_tiles, d->tb_ptr, d->tb_blk, d->blk_jk, d->sblk, d->na,
        nd ? d->slds : d->ld, nd ? d->nd_rhs : d->rhs, d->scal + 4, nd ? d->nd_crow : nullptr,
        nd ? d->nd_rowsrc : nullptr, d->rhs);
    return -(int)hipGetLastError();
}

int ba_chol_prepare(ba_dev *d)
{
    k_zero_env<<<d->n_env, 256, 0, d->stream>>>(d->S, d->lds, d->env_tiles);
    return -(int)hipGetLastError();
}

// the same rule on a dense ld x ld S (the natural-order retry of a
// nested-dissection pivot, ba_solver.cpp) and the camera-order rhs
int ba_fix_diag_plain(ba_dev *d, double *S, long long ld)
{
    k_fix_diag<<<(int)((ld + 255) / 256), 256, 0, d->stream>>>(S, d->rhs, ld);
    return -(int)hipGetLastError();
}

int ba_chol_fix_diag(ba_dev *d)
{
    k_fix_diag<<<(int)((d->lds + 255) / 256), 256, 0, d->stream>>>(d->S, d->rhs, d->lds);
    return -(int)hipGetLastError();
}

// runner mode (k_env_runner) for this factorization?  Needs the hand-off, the
// device panel pointers and the flags; off under per-kernel timing (one stream)
// and, for the rest of this context, after one of the runner's own hand-offs
// gave up (ba_env_runner_timed_out): the runner needs its side stream on a
// hardware queue of its own (with the library stream's column launches queued
// behind it on a shared queue every wait times out)
int ba_env_runner_timed_out(ba_dev *d)
{
    if (!d->env_runner || !d->rflag) return 0;
    unsigned *rto = d->rflag + 4 * (size_t)d->nt;
    unsigned h = 0;
    if (hipMemcpyAsync(&h, rto, sizeof h, hipMemcpyDeviceToHost, d->stream) != hipSuccess ||
        hipStreamSynchronize(d->stream) != hipSuccess)
        return -1;
    if (!h) return 0;
    d->env_runner = 0;
    std::fprintf(stderr, "[vlgba] envelope runner off for this context: one of its hand-offs "
                         "timed out (its stream shares a hardware queue?)\n");
    return 1;
}

// runs shorter than VLGBA_ENV_RUNNER_MIN columns (default 8) keep the column
// launches alone: the fork / join of the runner's stream (two cross-stream
// event waits a factorization) outweighs a few columns' savings (~3-5 us each)
static int env_run_min()
{
    const char *e = std::getenv("VLGBA_ENV_RUNNER_MIN");
    return e ? std::max(1, std::atoi(e)) : 8;
}

// the runner's stream: one per device for the process, at the highest
// priority, made on first use (a stream per context cost ~1 ms a context in
// the growing replay).  Two contexts factoring on one device at once
// serialise their runners; the later one's hand-offs may then give up (the
// re-solve path) -- correct, only slower.
static hipStream_t env_runner_stream()
{
    static std::mutex mu;
    static hipStream_t st[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!st[dev]) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (hipStreamCreateWithPriority(&st[dev], hipStreamNonBlocking, hi) != hipSuccess)
            st[dev] = nullptr;
    }
    return st[dev];
}

static bool env_run_on(ba_dev *d, const unsigned *kflag, int ncols)
{
    if (!(d->env_runner && kflag && d->pan_ptr && d->rflag && !(d->kt && d->kt->on) &&
          ncols >= env_run_min()))
        return false;
    if (!d->rstream) d->rstream = env_runner_stream();
    if (!d->rstream) {
        d->env_runner = 0;
        return false;
    }
    return true;
}

static env_rm env_rm_of(const ba_dev *d, int kend)
{
    if (!d->rflag) return env_rm{};
    return env_rm{d->rflag, d->rflag + d->nt, d->rflag + 2 * (size_t)d->nt,
                  d->rflag + 3 * (size_t)d->nt, d->rflag + 4 * (size_t)d->nt, kend};
}

// fork the side stream off the library stream and start the runner there.
// Nonzero: nothing was launched (the caller runs the column launches alone)
// or the launch failed (the error is returned).
static int env_runner_start(ba_dev *d, const env_runs &Rn, long long L, double *rhs)
{
    if (d->debug_runner_fail > 0) {   // vlgba_debug_force_status word 6
        d->debug_runner_fail--;
        return -(int)hipErrorLaunchFailure;
    }
    const size_t smem4 = sizeof(double) * 4 * NB * LP;
    TRY_RC(ba_ensure_dyn_lds((const void *)k_env_runner, smem4));
    VLGBA_CHECK(hipEventRecord(d->ev_fork, d->stream));
    VLGBA_CHECK(hipStreamWaitEvent(d->rstream, d->ev_fork, 0));
    k_env_runner<<<Rn.np, 256, smem4, d->rstream>>>(d->S, L, d->pan_ptr, d->pan_list, Rn,
                                                    d->linv, rhs, d->ywork, d->scal + 4,
                                                    d->kflag, env_rm_of(d, 0), d->fac_epoch);
    TRY_RC(-(int)hipGetLastError());
    VLGBA_CHECK(hipEventRecord(d->ev_join, d->rstream));
    d->runner_runs++;
    return 0;
}

// the envelope's tile columns k0 .. k1-1 (k_factor_step), column k0 taking no
// pending update of column k0-1.  A runner that does not start leaves the
// columns to the launches alone (the same factorization, bit for bit).
static int envelope_columns(ba_dev *d, int k0, int k1, long long L, double *rhs,
                            unsigned *kflag)
{
    // two LDS tiles with the hand-off (two workgroups per CU), three without
    const size_t smem3 = sizeof(double) * 3 * NB * LP, smem2 = sizeof(double) * 2 * NB * LP;
    bool run = k1 > k0 && env_run_on(d, kflag, k1 - k0);
    if (run) {
        env_runs Rn{};
        Rn.np = 1;
        Rn.k0[0] = k0;
        Rn.k1[0] = k1;
        if (env_runner_start(d, Rn, L, rhs)) run = false;
    }
    for (int k = k0; k < k1; k++) {
        const int p0 = d->pan_ptr_h[k], T = d->pan_ptr_h[k + 1] - p0;
        const int q0 = k > k0 ? d->pan_ptr_h[k - 1] : 0, Tp = k > k0 ? p0 - q0 : 0;
        // column k-1's trailing pairs below row k (see k_factor_step)
        const int kin = Tp > 0 && d->h_pan_list[q0] == k;
        const int Tr = Tp - kin, ntr = Tr * (Tr + 1) / 2;
        const int nw = ntr;   // one workgroup per trailing pair
        KT_B(d);
        k_factor_step<<<1 + T + nw, 256, kflag ? smem2 : smem3, d->stream>>>(
            d->S, L, k, d->pan_list + p0, T, d->pan_list + q0, Tp, d->linv, rhs, d->ywork,
            d->scal + 4, kflag, d->fac_epoch, ntr, nw, env_rm_of(d, run ? k1 : 0));
        KT_E(d, KT_FACTOR);
    }
    if (run) VLGBA_CHECK(hipStreamWaitEvent(d->stream, d->ev_join, 0));
    return -(int)hipGetLastError();
}

// x = L^-T y of the envelope factor (ywork holds y; consumed)
static int envelope_backward(ba_dev *d, long long L, double *x, int nospin)
{
    const int nt = d->nt;
    if (d->xgran64 && !nospin) {   // every column co-resident: the backward solve in one launch
        if (++d->back_epoch == 0) d->back_epoch = 1;
        const size_t smem2 = sizeof(double) * 2 * NB * LP;
        TRY_RC(ba_ensure_dyn_lds((const void *)k_backward_all, smem2));
        KT_B(d);
        k_backward_all<<<nt, 256, smem2, d->stream>>>(d->S, L, nt, d->pan_ptr, d->pan_list,
                                                       d->linv, d->ywork, x, d->xgran64,
                                                       d->back_epoch, d->scal + 4);
        KT_E(d, KT_BACKWARD);
        return -(int)hipGetLastError();
    }
    for (int k = nt - 1; k >= 0; k--) {
        const int j0 = d->h_tfirst[k];
        KT_B(d);
        k_backward<<<k - j0 + 1, 256, 0, d->stream>>>(d->S, L, k, j0, d->linv, d->ywork, x);
        KT_E(d, KT_BACKWARD);
    }
    return -(int)hipGetLastError();
}

int ba_chol_solve(ba_dev *d, int nospin)
{
    const int nt = d->nt;
    const size_t smem3 = sizeof(double) * 3 * NB * LP;
    TRY_RC(ba_ensure_dyn_lds((const void *)k_factor_step, smem3));
    TRY_RC(ba_ensure_dyn_lds((const void *)k_cr_factor, smem3));
    TRY_RC(ba_ensure_dyn_lds((const void *)k_cr_update, smem3));
    if (d->dense_solve == 3) {   // sequential parity solve
        KT_B(d);
        k_chol_seq<<<1, 256, 0, d->stream>>>(d->S, d->lds, (int)d->ld, d->rhs, d->da,
                                             d->scal + 4);
        KT_E(d, KT_FACTOR);
        return -(int)hipGetLastError();
    }
    if (d->cr_nlev > 0 && d->cr32 && d->cr_fused && d->crflag && !nospin) {   // one launch
        const int nl = d->cr_nlev, nrec = d->cr_eptr_h[nl];
        cr32_fplan P{};
        P.nl = nl;
        P.nrec = nrec;
        P.l0two = 3 * d->cr_eptr_h[1] > d->ncu;
        P.b0[0] = 0;
        P.b0[1] = (P.l0two ? 2 : 3) * d->cr_eptr_h[1];
        for (int l = 1; l < nl; l++) {
            const int nf = d->crf_ptr_h[l + 1] - d->crf_ptr_h[l];
            const int ns = d->crs_ptr_h[l + 1] - d->crs_ptr_h[l];
            P.fofs[l] = d->crf_ptr_h[l];
            P.sofs[l] = d->crs_ptr_h[l];
            P.b0[l + 1] = P.b0[l] + 3 * nf + ns;
        }
        P.sofs[nl] = d->crs_ptr_h[nl];
        for (int l = 0; l <= nl; l++) P.eofs[l] = d->cr_eptr_h[l];
        if (++d->back_epoch == 0) d->back_epoch = 1;
        KT_B(d);
        k_cr32_fused<<<P.b0[nl] + nrec, 256, 0, d->stream>>>(
            d->S, d->lds, d->tb32, d->ld, d->cr_elim, d->crf, d->crs, d->nt32, d->linv, d->crL,
            d->rhs, d->ywork, d->da, d->crflag, d->xgran, d->back_epoch, d->scal + 4, P);
        KT_E(d, KT_CR_FACTOR);
        return -(int)hipGetLastError();
    }
    if (d->cr_nlev > 0 && d->cr32) {   // camera-aligned 32-row tiles
        const int ncu32 = d->ncu;
        const int n32 = d->nt32, TB = d->tb32;
        {   // level 0 on the assembled S
            const int ne = d->cr_eptr_h[1];
            const int fs = 3 * ne <= 2 * ncu32;   // ~60 KB LDS: two workgroups per CU
            KT_B(d);
            k_cr32_factor<<<fs ? 3 * ne : ne, 256, 0, d->stream>>>(
                d->S, d->lds, TB, d->ld, d->cr_elim, n32, d->linv, d->crL, d->rhs, d->ywork,
                d->scal + 4, fs);
            KT_E(d, KT_CR_FACTOR);
        }
        // levels >= 1: the previous level's update folded into the factor launch
        for (int l = 1; l < d->cr_nlev; l++) {
            const int f0 = d->crf_ptr_h[l], ne = d->crf_ptr_h[l + 1] - f0;
            const int s0 = d->crs_ptr_h[l], ns = d->crs_ptr_h[l + 1] - s0;
            KT_B(d);
            k_cr32_level<<<3 * ne + ns, 256, 0, d->stream>>>(
                d->S, d->lds, TB, d->ld, d->crf + 5 * f0, ne, d->crs + 3 * s0, n32, d->linv,
                d->crL, d->rhs, d->ywork, d->scal + 4);
            KT_E(d, KT_CR_FACTOR);
        }
        const int nrec = d->cr_eptr_h[d->cr_nlev];
        if (d->xgran && nrec <= 2 * d->ncu && !nospin) {   // every record co-resident: one launch
            if (++d->back_epoch == 0) d->back_epoch = 1;
            KT_B(d);
            k_cr32_back_all<<<nrec, 256, 0, d->stream>>>(d->cr_elim, nrec, n32, TB, d->ld,
                                                         d->linv, d->crL, d->ywork, d->da,
                                                         d->xgran, d->back_epoch, d->scal + 4);
            KT_E(d, KT_CR_BACK);
            return -(int)hipGetLastError();
        }
        for (int l = d->cr_nlev - 1; l >= 0; l--) {
            const int e0 = d->cr_eptr_h[l], ne = d->cr_eptr_h[l + 1] - e0;
            KT_B(d);
            k_cr32_back<<<ne, 256, 0, d->stream>>>(d->cr_elim + 3 * e0, n32, TB, d->ld,
                                                   d->linv, d->crL, d->ywork, d->da);
            KT_E(d, KT_CR_BACK);
        }
        return -(int)hipGetLastError();
    }
    if (d->cr_nlev > 0) {   // (status cleared by k_assemble_tiles)
        // one workgroup per CU (LDS): fan a level out over 5 (factor) / 4
        // (update) workgroups per tile while that still fits in one wave of
        // workgroups -- the levels are latency bound, the chip mostly idle
        const int ncu = d->ncu;
        for (int l = 0; l < d->cr_nlev; l++) {
            const int e0 = d->cr_eptr_h[l], ne = d->cr_eptr_h[l + 1] - e0;
            const int k0 = d->cr_kptr_h[l], nk = d->cr_kptr_h[l + 1] - k0;
            const int fs = 5 * ne <= ncu, us = 4 * nk <= ncu;
            KT_B(d);
            k_cr_factor<<<fs ? 5 * ne : ne, 256, smem3, d->stream>>>(
                d->S, d->lds, d->cr_elim + 3 * e0, nt, d->linv, d->crL, d->rhs, d->ywork,
                d->scal + 4, fs);
            KT_E(d, KT_CR_FACTOR);
            if (nk > 0) {
                KT_B(d);
                k_cr_update<<<us ? 4 * nk : nk, 256, smem3, d->stream>>>(
                    d->S, d->lds, d->cr_keep + 4 * k0, nt, d->crL, d->rhs, d->ywork, us);
                KT_E(d, KT_CR_UPDATE);
            }
        }
        for (int l = d->cr_nlev - 1; l >= 0; l--) {
            const int e0 = d->cr_eptr_h[l], ne = d->cr_eptr_h[l + 1] - e0;
            KT_B(d);
            k_cr_back<<<ne, 256, 0, d->stream>>>(d->cr_elim + 3 * e0, nt, d->linv, d->crL,
                                                 d->ywork, d->da);
            KT_E(d, KT_CR_BACK);
        }
        return -(int)hipGetLastError();
    }
    // the envelope factor's in-launch hand-off (not in a re-solve)
    unsigned *kflag = nospin ? nullptr : d->kflag;
    if (kflag && ++d->fac_epoch == 0) d->fac_epoch = 1;
    if (d->nd_np > 0) {   // nested dissection: the arcs side by side, then the separator
        const int np = d->nd_np, s0 = d->nd_a0[np];
        const long long L = d->slds;
        TRY_RC(ba_ensure_dyn_lds((const void *)k_factor_multi, smem3));
        int nsteps = 0;
        for (int t = 0; t < np; t++) nsteps = std::max(nsteps, d->nd_a0[t + 1] - d->nd_a0[t]);
        bool run = env_run_on(d, kflag, nsteps);
        if (run) {
            env_runs Rn{};
            Rn.np = np;
            for (int t = 0; t < np; t++) {
                Rn.k0[t] = d->nd_a0[t];
                Rn.k1[t] = d->nd_a0[t + 1];
            }
            if (env_runner_start(d, Rn, L, d->nd_rhs)) run = false;   // the launches alone
        }
        for (int st = 0; st < nsteps; st++) {
            nd_step P{};
            P.grouped = d->nd_grouped;
            int nbk = 0;
            for (int t = 0; t < np; t++) {
                const int k = d->nd_a0[t] + st;
                if (k >= d->nd_a0[t + 1]) continue;
                const int p0 = d->pan_ptr_h[k], T = d->pan_ptr_h[k + 1] - p0;
                const bool cont = k > d->nd_a0[t];   // not the arc's first column
                const int q0 = cont ? d->pan_ptr_h[k - 1] : 0, Tp = cont ? p0 - q0 : 0;
                const int kin = Tp > 0 && d->h_pan_list[q0] == k;
                int nsr = 0;   // separator rows among column k-1's trailing rows
                for (int q = q0 + kin; q < q0 + Tp; q++) nsr += d->h_pan_list[q] >= s0;
                const int Tr = Tp - kin, u = P.np++;
                P.k[u] = k;
                P.T[u] = T;
                P.Tp[u] = Tp;
                P.pofs[u] = p0;
                P.qofs[u] = q0;
                const int ntr = Tr * (Tr + 1) / 2 - nsr * (nsr + 1) / 2;
                P.ntr[u] = ntr;
                P.kend[u] = run ? d->nd_a0[t + 1] : 0;
                P.b0[u] = nbk;
                P.pb[u + 1] = P.pb[u] + T;
                nbk += 1 + T;
            }
            // the trailing workgroups: each arc's share of the cap (with the hand-off)
            int ttot = 0;
            for (int u = 0; u < P.np; u++) ttot += P.ntr[u];
            const int tw = ttot;   // one workgroup per trailing pair
            for (int u = 0; u < P.np; u++) {
                const int nw = tw == ttot ? P.ntr[u]
                                          : (P.ntr[u] == 0 ? 0
                                                           : std::max(1, (int)((long long)tw *
                                                                               P.ntr[u] / ttot)));
                P.ts[u] = nw;
                P.tb[u + 1] = P.tb[u] + nw;
            }
            if (!P.grouped) {   // arc-major: arc u's trailing workgroups follow its panels
                int acc = 0;
                for (int u = 0; u < P.np; u++) {
                    P.b0[u] = acc;
                    acc += 1 + P.T[u] + P.ts[u];
                }
            }
            nbk += P.tb[P.np];
            P.b0[P.np] = nbk;
            KT_B(d);
            k_factor_multi<<<nbk, 256, kflag ? sizeof(double) * 2 * NB * LP : smem3, d->stream>>>(
                d->S, L, d->pan_list, P, s0, d->linv,
                                                          d->nd_rhs, d->ywork, d->scal + 4, kflag,
                                                          d->fac_epoch, env_rm_of(d, 0));
            KT_E(d, KT_FACTOR);
        }
        if (run) VLGBA_CHECK(hipStreamWaitEvent(d->stream, d->ev_join, 0));
        if (d->nd_nrec > 0) {
            const size_t smem2 = sizeof(double) * 2 * NB * LP;
            TRY_RC(ba_ensure_dyn_lds((const void *)k_sep_update, smem2));
            KT_B(d);
            k_sep_update<<<d->nd_nrec, 256, smem2, d->stream>>>(
                d->S, L, d->nd_pair, d->nd_rec, d->nd_klist, d->ywork, d->nd_part);
            k_sep_reduce<<<d->nd_npair, 256, 0, d->stream>>>(d->S, L, d->nd_pair, d->nd_pptr,
                                                             d->nd_part, d->nd_rhs);
            KT_E(d, KT_SYRK);
        }
        TRY_RC(envelope_columns(d, s0, nt, L, d->nd_rhs, kflag));
        TRY_RC(envelope_backward(d, L, d->nd_x, nospin));
        k_nd_scatter<<<(int)((d->lds + 255) / 256), 256, 0, d->stream>>>(d->nd_prow, d->nd_x,
                                                                         d->da, d->lds);
        return -(int)hipGetLastError();
    }
    TRY_RC(envelope_columns(d, 0, nt, d->lds, d->rhs, kflag));
    TRY_RC(envelope_backward(d, d->lds, d->da, nospin));
    return -(int)hipGetLastError();
}
