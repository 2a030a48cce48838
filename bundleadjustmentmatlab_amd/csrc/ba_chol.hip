// ba_chol.hip -- dense reduced-camera solve on gfx950: blocked right-looking
// Cholesky with fp64 MFMA (v_mfma_f64_16x16x4_f64) + triangular solves.
//
// Replaces da = pinv(S) * e_ (toolbox/bundle/bundle_euclid.m:193).  S is
// symmetric positive definite once its exactly-zero rows (fixed parameters,
// App. A Q2/Q8) have been replaced by identity rows in k_fix_zero_rows, and on
// that matrix pinv and the Cholesky solve agree to conditioning-limited
// rounding.  A non-positive pivot sets *status (the host then treats the step
// like a rejected one).
//
// Storage: S column major, leading dimension lds (a multiple of NB = 64),
// lower triangle used.  Per tile column k:
//   k_potrf_tile : factor L_kk in LDS, form L_kk^-1 (kept per k for the
//                  backward solve), y_k = L_kk^-1 r_k  (forward solve folded in)
//   k_panel      : L_ik = A_ik L_kk^-T as an MFMA GEMM against L_kk^-1, then
//                  r_i -= L_ik y_k
//   k_syrk       : A_ij -= L_ik L_jk^T for k < j <= i (MFMA), the bulk
// then per k descending k_backward: x_k = L_kk^-T z_k, z_j -= L_kj^T x_k.
#include "ba_internal.h"

#define NB 64
#define LP 66  // LDS row pitch in doubles: lanes r and r+1 / t and t+1 of a
               // 16x4 MFMA operand read land on distinct ds_read_b64 banks

typedef double d4 __attribute__((ext_vector_type(4)));

// load tile (ti, tj) of S (column major) into LDS row-major T[r][c]
__device__ __forceinline__ void load_tile(const double *__restrict__ S, long long lds, int ti,
                                          int tj, double *T)
{
    const double *base = S + (long long)NB * ti + lds * (long long)NB * tj;
    for (int q = threadIdx.x; q < NB * NB; q += blockDim.x) {
        const int r = q & (NB - 1), c = q >> 6;
        T[r * LP + c] = base[r + lds * c];
    }
}

// acc(64x64 per workgroup of 256) = As[r][:] . Bs[c][:]  (both row-major, K = 64)
// wave w owns rows 32*(w>>1) .. +31 and cols 32*(w&1) .. +31 as 2x2 MFMA tiles.
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

// ---------------------------------------------------------------------------
// diagonal tile: Cholesky in LDS, explicit inverse, forward-solve step
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf_tile(double *__restrict__ S, long long lds, int k,
                                                    double *__restrict__ linv,
                                                    const double *__restrict__ rhs,
                                                    double *__restrict__ y,
                                                    double *__restrict__ status)
{
    __shared__ double A[NB * LP];
    __shared__ double Li[NB * LP];
    __shared__ double piv;
    const int tid = threadIdx.x;
    load_tile(S, lds, k, k, A);
    __syncthreads();
    for (int c = 0; c < NB; c++) {
        if (tid == 0) {
            double d = A[c * LP + c];
            if (!(d > 0.0)) {
                status[0] = 1.0;
                d = 1.0;
            }
            piv = sqrt(d);
            A[c * LP + c] = piv;
        }
        __syncthreads();
        const double p = piv;
        if (tid > c && tid < NB) A[tid * LP + c] = A[tid * LP + c] / p;
        __syncthreads();
        // trailing update of the tile's lower triangle
        const int rem = NB - 1 - c;
        for (int q = tid; q < rem * rem; q += blockDim.x) {
            const int r = c + 1 + q / rem, cc = c + 1 + q % rem;
            if (cc <= r) A[r * LP + cc] -= A[r * LP + c] * A[cc * LP + c];
        }
        __syncthreads();
    }
    // write L_kk (lower) back; zero the strict upper part of the tile
    {
        double *base = S + (long long)NB * k + lds * (long long)NB * k;
        for (int q = tid; q < NB * NB; q += blockDim.x) {
            const int r = q & (NB - 1), c = q >> 6;
            base[r + lds * c] = (r >= c) ? A[r * LP + c] : 0.0;
        }
    }
    // Li = L^-1 (lower): thread c solves L x = e_c by forward substitution
    if (tid < NB) {
        const int c = tid;
        for (int r = 0; r < c; r++) Li[r * LP + c] = 0.0;
        Li[c * LP + c] = 1.0 / A[c * LP + c];
        for (int r = c + 1; r < NB; r++) {
            double s = 0.0;
            for (int q = c; q < r; q++) s += A[r * LP + q] * Li[q * LP + c];
            Li[r * LP + c] = -s / A[r * LP + r];
        }
    }
    __syncthreads();
    double *lo = linv + (long long)NB * NB * k;
    for (int q = tid; q < NB * NB; q += blockDim.x) {
        const int r = q >> 6, c = q & (NB - 1);
        lo[q] = Li[r * LP + c];  // row-major L^-1
    }
    // y_k = L_kk^-1 r_k
    if (tid < NB) {
        double s = 0.0;
        for (int q = 0; q <= tid; q++) s += Li[tid * LP + q] * rhs[(long long)NB * k + q];
        y[(long long)NB * k + tid] = s;
    }
}

// ---------------------------------------------------------------------------
// panel: L_ik = A_ik L_kk^-T, r_i -= L_ik y_k   (grid: i = k+1 .. nt-1)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_panel(double *__restrict__ S, long long lds, int k,
                                               const double *__restrict__ linv,
                                               double *__restrict__ rhs,
                                               const double *__restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    const int i = k + 1 + blockIdx.x;
    const int tid = threadIdx.x;
    load_tile(S, lds, i, k, As);
    const double *lo = linv + (long long)NB * NB * k;
    for (int q = tid; q < NB * NB; q += blockDim.x) Bs[(q >> 6) * LP + (q & 63)] = lo[q];
    __syncthreads();
    d4 acc[2][2];
    mfma_64x64(As, Bs, acc);
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    double *base = S + (long long)NB * i + lds * (long long)NB * k;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int yy = 0; yy < 2; yy++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = r0 + 16 * x + (lane >> 4) + 4 * q, c = c0 + 16 * yy + (lane & 15);
                As[r * LP + c] = acc[x][yy][q];
                base[r + lds * c] = acc[x][yy][q];
            }
    __syncthreads();
    if (tid < NB) {
        double s = 0.0;
        for (int c = 0; c < NB; c++) s += As[tid * LP + c] * y[(long long)NB * k + c];
        rhs[(long long)NB * i + tid] -= s;
    }
}

// ---------------------------------------------------------------------------
// trailing update A_ij -= L_ik L_jk^T, k < j <= i   (grid: lower tiles)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_syrk(double *__restrict__ S, long long lds, int k, int nt)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    // blockIdx.x -> (i, j) over the lower triangle of the (nt-k-1)^2 trailing tiles
    const int T = nt - k - 1;
    int q = blockIdx.x, jj = 0;
    while (q >= T - jj) { q -= T - jj; jj++; }
    const int j = k + 1 + jj, i = j + q;
    (void)T;
    load_tile(S, lds, i, k, As);
    load_tile(S, lds, j, k, Bs);
    __syncthreads();
    d4 acc[2][2];
    mfma_64x64(As, Bs, acc);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
    double *base = S + (long long)NB * i + lds * (long long)NB * j;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int yy = 0; yy < 2; yy++)
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const int r = r0 + 16 * x + (lane >> 4) + 4 * qq, c = c0 + 16 * yy + (lane & 15);
                base[r + lds * c] -= acc[x][yy][qq];
            }
}

// ---------------------------------------------------------------------------
// backward solve step k: x_k = L_kk^-T z_k; z_j -= L_kj^T x_k (grid j = 0..k)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_backward(const double *__restrict__ S, long long lds,
                                                  int k, const double *__restrict__ linv,
                                                  double *__restrict__ z, double *__restrict__ x)
{
    __shared__ double xs[NB];
    __shared__ double part[4][NB];
    const int j = blockIdx.x, tid = threadIdx.x;
    const double *lo = linv + (long long)NB * NB * k;  // row-major L^-1
    if (tid < NB) {
        double s = 0.0;
        for (int r = tid; r < NB; r++) s += lo[r * NB + tid] * z[(long long)NB * k + r];
        xs[tid] = s;
    }
    __syncthreads();
    if (j == k) {
        if (tid < NB) x[(long long)NB * k + tid] = xs[tid];
        return;
    }
    // z_j[c] -= sum_r L_kj[r][c] x_k[r]; 4 partial sums over row quarters
    const int c = tid & 63, qr = tid >> 6;
    const double *base = S + (long long)NB * k + lds * (long long)NB * j;
    double s = 0.0;
    for (int r = 16 * qr; r < 16 * qr + 16; r++) s += base[r + lds * c] * xs[r];
    part[qr][c] = s;
    __syncthreads();
    if (tid < NB)
        z[(long long)NB * j + tid] -= ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
}

int ba_chol_solve(ba_dev *d)
{
    const int nt = (int)(d->lds / NB);
    const size_t smem = sizeof(double) * 2 * NB * LP;
    static bool attr_done = false;
    if (!attr_done) {
        VLGBA_CHECK(hipFuncSetAttribute((const void *)k_panel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        VLGBA_CHECK(hipFuncSetAttribute((const void *)k_syrk,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
        attr_done = true;
    }
    VLGBA_CHECK(hipMemsetAsync(d->scal + 4, 0, sizeof(double), d->stream));
    for (int k = 0; k < nt; k++) {
        k_potrf_tile<<<1, 256, 0, d->stream>>>(d->S, d->lds, k, d->linv, d->rhs, d->ywork,
                                               d->scal + 4);
        const int T = nt - k - 1;
        if (T > 0) {
            k_panel<<<T, 256, smem, d->stream>>>(d->S, d->lds, k, d->linv, d->rhs, d->ywork);
            k_syrk<<<T * (T + 1) / 2, 256, smem, d->stream>>>(d->S, d->lds, k, nt);
        }
    }
    for (int k = nt - 1; k >= 0; k--)
        k_backward<<<k + 1, 256, 0, d->stream>>>(d->S, d->lds, k, d->linv, d->ywork, d->da);
    return -(int)hipGetLastError();
}
