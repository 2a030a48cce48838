// ba_chol.hip -- dense reduced-camera solve on gfx950: blocked right-looking
// tile Cholesky with fp64 MFMA (v_mfma_f64_16x16x4_f64) + triangular solves.
//
// Replaces da = pinv(S) * e_ (toolbox/bundle/bundle_euclid.m:193).  S is
// symmetric positive definite once its exactly-zero rows (fixed parameters,
// App. A Q2/Q8) are given a unit diagonal (k_fix_diag), and on that matrix
// pinv and the Cholesky solve agree to conditioning-limited rounding.  A
// non-positive pivot sets *status (the host treats the step as rejected).
//
// Storage: S column major, leading dimension lds (multiple of NB = 64), lower
// triangle.  Tile envelope: tile row i of S (hence of L: the profile is
// preserved by Cholesky) is zero left of tile column tfirst[i]; every kernel
// below visits only tiles inside the envelope, which is exact (the skipped
// tiles are zero and stay zero).  dense_solve = 1 visits every lower tile.
//
// Per tile column k (two launches):
//   k_factor_panel : WG 0 factors L_kk in registers (one wave), forms
//                    L_kk^-1 and y_k = L_kk^-1 r_k (forward solve folded in);
//                    WG b >= 1 redoes that factorisation in LDS and computes
//                    panel tile L_ik = A_ik L_kk^-T (MFMA), r_i -= L_ik y_k
//   k_syrk         : A_ij -= L_ik L_jk^T for envelope pairs k < j <= i (MFMA)
// then per k descending k_backward: x_k = L_kk^-T z_k, z_j -= L_kj^T x_k.
#include "ba_internal.h"

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
__device__ __forceinline__ void mfma_64x64(const double *As, const double *Bs, d4 acc[2][2])
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
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

// The whole 256-thread workgroup factors the 64x64 SPD tile in As (row-major,
// lower used) and inverts the factor in the same right-looking sweep:
// thread (r = tid & 63, g = tid >> 6) keeps row r, columns 16g .. 16g+15 of A
// and of X (X starts as I; solving L X = I row by row gives X = L^-1).
// Column c of L and row c of X are broadcast through LDS (double-buffered by
// the parity of c: two barriers per column).  Writes L (zero upper) to As and
// L^-1 to Li (both row-major).  Returns false on a non-positive pivot.
__device__ bool block_potrf_inv(double *As, double *Li)
{
    __shared__ double colL[2][NB];
    __shared__ double rowX[2][NB];
    __shared__ double rpiv[2];
    __shared__ int bad;
    const int tid = threadIdx.x, r = tid & 63, g = tid >> 6;
    double a[16], x[16];
#pragma unroll
    for (int jj = 0; jj < 16; jj++) {
        a[jj] = As[r * LP + 16 * g + jj];
        x[jj] = (r == 16 * g + jj) ? 1.0 : 0.0;
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int gc = 0; gc < 4; gc++)
#pragma unroll
    for (int jc = 0; jc < 16; jc++) {
        const int c = 16 * gc + jc, b = jc & 1;
        if (g == gc && r == c) {
            double d = a[jc];
            if (!(d > 0.0)) {
                bad = 1;
                d = 1.0;
            }
            a[jc] = sqrt(d);
            colL[b][c] = a[jc];
            rpiv[b] = 1.0 / a[jc];     // one division per column; scale by it
        }
        __syncthreads();
        const double rp = rpiv[b];
        if (g == gc && r > c) {
            a[jc] = a[jc] * rp;
            colL[b][r] = a[jc];
        }
        if (r == c) {
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                x[jj] = x[jj] * rp;
                rowX[b][16 * g + jj] = x[jj];
            }
        }
        __syncthreads();
        if (r > c) {
            const double lrc = colL[b][r];
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                const int q = 16 * g + jj;
                if (q > c && q <= r) a[jj] = fma(-lrc, colL[b][q], a[jj]);
                x[jj] = fma(-lrc, rowX[b][q], x[jj]);
            }
        }
    }
#pragma unroll
    for (int jj = 0; jj < 16; jj++) {
        const int q = 16 * g + jj;
        As[r * LP + q] = (q <= r) ? a[jj] : 0.0;
        Li[r * LP + q] = x[jj];
    }
    __syncthreads();
    return bad == 0;
}

// ---------------------------------------------------------------------------
// factor + panel for tile column k.  blockIdx 0: diagonal; b >= 1: panel tile
// pan[b-1].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_factor_panel(double *__restrict__ S, long long lds,
                                                      int k, const int *__restrict__ pan,
                                                      double *__restrict__ linv,
                                                      double *__restrict__ rhs,
                                                      double *__restrict__ y,
                                                      double *__restrict__ status)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    __shared__ double yk[NB], rk[NB];
    const int tid = threadIdx.x;
    load_tile(S, lds, k, k, As);
    if (tid < NB) rk[tid] = rhs[(long long)NB * k + tid];
    __syncthreads();
    const bool ok = block_potrf_inv(As, Bs);
    // y_k = L^-1 r_k
    if (tid < NB) {
        double s = 0.0;
        for (int q = 0; q <= tid; q++) s += Bs[tid * LP + q] * rk[q];
        yk[tid] = s;
    }
    if (blockIdx.x == 0) {
        store_tile(S, lds, k, k, As);
        double *lo = linv + (long long)NB * NB * k;
        for (int q = tid; q < NB * NB; q += blockDim.x) lo[q] = Bs[(q >> 6) * LP + (q & 63)];
        __syncthreads();
        if (tid < NB) y[(long long)NB * k + tid] = yk[tid];
        if (tid == 0 && !ok) status[0] = 1.0;
        return;
    }
    const int i = pan[blockIdx.x - 1];
    __syncthreads();
    load_tile(S, lds, i, k, As);
    __syncthreads();
    d4 acc[2][2];
    mfma_64x64(As, Bs, acc);   // L_ik[r][c] = sum_t A_ik[r][t] Li[c][t]
    __syncthreads();
    acc_to_lds(acc, As, 1.0, false);
    __syncthreads();
    store_tile(S, lds, i, k, As);
    if (tid < NB) {
        double s = 0.0;
        for (int c = 0; c < NB; c++) s += As[tid * LP + c] * yk[c];
        rhs[(long long)NB * i + tid] -= s;
    }
}

// ---------------------------------------------------------------------------
// trailing update A_ij -= L_ik L_jk^T for pan pairs (jj <= ii)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_syrk(double *__restrict__ S, long long lds, int k,
                                              const int *__restrict__ pan, int T)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    int q = blockIdx.x, jj = 0;
    while (q >= T - jj) {
        q -= T - jj;
        jj++;
    }
    const int j = pan[jj], i = pan[jj + q];
    load_tile(S, lds, i, k, As);
    load_tile(S, lds, j, k, Bs);
    __syncthreads();
    d4 acc[2][2];
    mfma_64x64(As, Bs, acc);
    __syncthreads();
    load_tile(S, lds, i, j, As);
    __syncthreads();
    acc_to_lds(acc, As, -1.0, true);
    __syncthreads();
    store_tile(S, lds, i, j, As);
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

// ===========================================================================
int ba_chol_setup(ba_dev *d, const int *blk_jk, int nb)
{
    const int nt = (int)(d->lds / NB);
    d->nt = nt;
    d->h_tfirst = new int[nt];
    for (int i = 0; i < nt; i++) d->h_tfirst[i] = d->dense_solve ? 0 : i;
    if (!d->dense_solve)
        for (int b = 0; b < nb; b++) {
            const int j = blk_jk[2 * b], k = blk_jk[2 * b + 1];   // j >= k
            const long long r0 = (long long)d->na * j, c0 = (long long)d->na * k;
            for (long long r = r0; r < r0 + d->na; r++) {
                const int ti = (int)(r / NB);
                const int tk = (int)(c0 / NB);
                if (tk < d->h_tfirst[ti]) d->h_tfirst[ti] = tk;
            }
        }
    std::vector<int> ptr(nt + 1, 0), list, env;
    for (int k = 0; k < nt; k++) {
        for (int i = k + 1; i < nt; i++)
            if (d->h_tfirst[i] <= k) list.push_back(i);
        ptr[k + 1] = (int)list.size();
    }
    for (int k = 0; k < nt; k++)
        for (int i = k; i < nt; i++)
            if (d->h_tfirst[i] <= k) {
                env.push_back(i);
                env.push_back(k);
            }
    d->n_env = (int)env.size() / 2;
    d->pan_ptr_h = new int[nt + 1];
    for (int k = 0; k <= nt; k++) d->pan_ptr_h[k] = ptr[k];
    VLGBA_CHECK(hipMalloc(&d->pan_list, sizeof(int) * (list.size() + 1)));
    VLGBA_CHECK(hipMalloc(&d->env_tiles, sizeof(int) * (env.size() + 1)));
    if (!list.empty())
        VLGBA_CHECK(hipMemcpyAsync(d->pan_list, list.data(), sizeof(int) * list.size(),
                                   hipMemcpyHostToDevice, d->stream));
    VLGBA_CHECK(hipMemcpyAsync(d->env_tiles, env.data(), sizeof(int) * env.size(),
                               hipMemcpyHostToDevice, d->stream));
    VLGBA_CHECK(hipMemsetAsync(d->S, 0, sizeof(double) * d->lds * d->lds, d->stream));
    VLGBA_CHECK(hipStreamSynchronize(d->stream));
    return 0;
}

void ba_chol_free(ba_dev *d)
{
    delete[] d->h_tfirst;
    delete[] d->pan_ptr_h;
    if (d->pan_list) (void)hipFree(d->pan_list);
    if (d->env_tiles) (void)hipFree(d->env_tiles);
    d->h_tfirst = d->pan_ptr_h = nullptr;
    d->pan_list = d->env_tiles = nullptr;
}

int ba_chol_prepare(ba_dev *d)
{
    k_zero_env<<<d->n_env, 256, 0, d->stream>>>(d->S, d->lds, d->env_tiles);
    return -(int)hipGetLastError();
}

int ba_chol_fix_diag(ba_dev *d)
{
    k_fix_diag<<<(int)((d->lds + 255) / 256), 256, 0, d->stream>>>(d->S, d->rhs, d->lds);
    return -(int)hipGetLastError();
}

int ba_chol_solve(ba_dev *d)
{
    const int nt = d->nt;
    const size_t smem = sizeof(double) * 2 * NB * LP;
    static bool attr_done = false;
    if (!attr_done) {
        VLGBA_CHECK(hipFuncSetAttribute((const void *)k_factor_panel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        VLGBA_CHECK(hipFuncSetAttribute((const void *)k_syrk,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        attr_done = true;
    }
    VLGBA_CHECK(hipMemsetAsync(d->scal + 4, 0, sizeof(double), d->stream));
    for (int k = 0; k < nt; k++) {
        const int p0 = d->pan_ptr_h[k], T = d->pan_ptr_h[k + 1] - p0;
        k_factor_panel<<<1 + T, 256, smem, d->stream>>>(d->S, d->lds, k, d->pan_list + p0,
                                                         d->linv, d->rhs, d->ywork,
                                                         d->scal + 4);
        if (T > 0)
            k_syrk<<<T * (T + 1) / 2, 256, smem, d->stream>>>(d->S, d->lds, k, d->pan_list + p0,
                                                              T);
    }
    for (int k = nt - 1; k >= 0; k--) {
        const int j0 = d->h_tfirst[k];
        k_backward<<<k - j0 + 1, 256, 0, d->stream>>>(d->S, d->lds, k, j0, d->linv, d->ywork,
                                                       d->da);
    }
    return -(int)hipGetLastError();
}
