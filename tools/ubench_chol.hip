// Diagnostic micro-benchmark of the Cholesky tile kernels (not part of the
// library).  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -I include -I bundleadjustmentmatlab_amd/csrc tools/ubench_chol.hip -o ubench_chol
// Prints in-kernel cycle stamps of the phases of block_potrf_inv and the
// wall time of k_factor_step on a 2-tile SPD matrix.
#include "../bundleadjustmentmatlab_amd/csrc/ba_chol.hip"

// the library's kernel-timer hooks (ba_solver.cpp) are not linked here
void kt_begin(ba_ktimer *, hipStream_t) {}
void kt_end(ba_ktimer *, hipStream_t, int) {}
// the library's caching allocator (ba_solver.cpp) is not linked here either
void *ba_dmalloc(size_t bytes)
{
    void *p = nullptr;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}
void ba_dfree(void *p) { (void)hipFree(p); }
int ba_ensure_dyn_lds(const void *fn, size_t bytes)
{
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) ==
                   hipSuccess ? 0 : -1;
}

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ unsigned long long stamp()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// copy of wave_factor16 with stamps: [0] pivot loop, [1] LDS write, [2] inverse
__device__ void wave_factor16_dbg(double *As, double *Bs, int o, unsigned long long *ts)
{
    const int r = threadIdx.x & 63;
    double d[16], rd[16];
#pragma unroll
    for (int c = 0; c < 16; c++) d[c] = (r < 16) ? As[(o + r) * LP + o + c] : 0.0;
    unsigned long long t0 = stamp();
#pragma unroll
    for (int c = 0; c < 16; c++) {
        double piv = rdlane(d[c], c);
        if (!(piv > 0.0)) piv = 1.0;
        double y = __builtin_amdgcn_rsq(piv);
        const double hp = 0.5 * piv;
        y = y * fma(-hp * y, y, 1.5);
        y = y * fma(-hp * y, y, 1.5);
        y = y * fma(-hp * y, y, 1.5);
        rd[c] = y;
        d[c] = (r == c) ? piv * y : ((r > c) ? d[c] * y : 0.0);
#pragma unroll
        for (int q = c + 1; q < 16; q++) d[q] = fma(-d[c], rdlane(d[c], q), d[q]);
    }
    asm volatile("" ::"v"(d[15]));
    unsigned long long t1 = stamp();
    if (r < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) As[(o + r) * LP + o + c] = (c <= r) ? d[c] : 0.0;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    unsigned long long t2 = stamp();
    double x[16];
#pragma unroll
    for (int q = 0; q < 16; q++) x[q] = (q == r) ? 1.0 : 0.0;
#pragma unroll
    for (int t = 0; t < 16; t++) {
        x[t] = x[t] * rd[t];
#pragma unroll
        for (int q = t + 1; q < 16; q++) x[q] = fma(-As[(o + q) * LP + o + t], x[t], x[q]);
    }
    if (r < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) Bs[(o + c) * LP + o + r] = x[c];
    }
    unsigned long long t3 = stamp();
    ts[0] = t1 - t0;
    ts[1] = t2 - t1;
    ts[2] = t3 - t2;
}

__global__ __launch_bounds__(256) void k_f16(const double *S, long long lds,
                                             unsigned long long *out)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    load_tile(S, lds, 0, 0, As);
    __syncthreads();
    unsigned long long ts[3];
    if (threadIdx.x < 64) wave_factor16_dbg(As, Bs, 0, ts);
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; q++) out[4 + q] = ts[q];
}

__global__ __launch_bounds__(256) void k_diag(const double *S, long long lds,
                                              unsigned long long *out)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    unsigned long long t0 = stamp();
    load_tile(S, lds, 0, 0, As);
    __syncthreads();
    unsigned long long t1 = stamp();
    // phase split of block_potrf_inv: factor16 only, on wave 0
    if (threadIdx.x < 64) wave_factor16(As, Bs, 0);
    __syncthreads();
    unsigned long long t2 = stamp();
    load_tile(S, lds, 0, 0, As);
    __syncthreads();
    unsigned long long t3 = stamp();
    block_potrf_inv(As, Bs);
    unsigned long long t4 = stamp();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = t2 - t1;
        out[2] = t4 - t3;
    }
}

int main()
{
    const int n = 128;
    std::vector<double> h((size_t)n * n);
    srand(1);
    std::vector<double> M((size_t)n * n);
    for (auto &v : M) v = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double s = (i == j) ? n : 0.0;
            for (int k = 0; k < n; k++) s += M[i * n + k] * M[j * n + k];
            h[i + (size_t)n * j] = s;
        }
    double *S, *S0, *linv, *rhs, *y, *st;
    int *pan;
    unsigned long long *out;
    hipMalloc(&S, sizeof(double) * n * n);
    hipMalloc(&S0, sizeof(double) * n * n);
    hipMalloc(&linv, sizeof(double) * 2 * 64 * 64);
    hipMalloc(&rhs, sizeof(double) * n);
    hipMalloc(&y, sizeof(double) * n);
    hipMalloc(&st, sizeof(double) * 4);
    hipMalloc(&pan, sizeof(int) * 4);
    hipMalloc(&out, sizeof(unsigned long long) * 8);
    hipMemcpy(S0, h.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    hipMemset(rhs, 0, sizeof(double) * n);
    int one = 1;
    hipMemcpy(pan, &one, sizeof(int), hipMemcpyHostToDevice);
    const size_t smem3 = sizeof(double) * 3 * NB * LP;
    hipFuncSetAttribute((const void *)k_factor_step, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    hipFuncSetAttribute((const void *)k_diag, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    k_diag<<<1, 256, smem3>>>(S0, n, out);
    unsigned long long ho[8];
    hipMemcpy(ho, out, sizeof(ho), hipMemcpyDeviceToHost);
    printf("cycles: load_tile %llu  factor16 %llu  block_potrf_inv %llu\n", ho[0], ho[1], ho[2]);
    hipFuncSetAttribute((const void *)k_f16, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    k_f16<<<1, 256, smem3>>>(S0, n, out);
    hipMemcpy(ho, out, sizeof(ho), hipMemcpyDeviceToHost);
    printf("factor16 parts: pivot loop %llu  lds write %llu  inverse %llu\n", ho[4], ho[5], ho[6]);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int fuse = 0; fuse < 2; fuse++) {
        float best = 1e9;
        for (int it = 0; it < 20; it++) {
            hipMemcpy(S, S0, sizeof(double) * n * n, hipMemcpyDeviceToDevice);
            hipEventRecord(e0);
            k_factor_step<<<2, 256, smem3>>>(S, n, 0, pan, 1, pan, 0, linv, rhs, y, st);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("k_factor_step (run %d): best %.2f us\n", fuse, best * 1e3);
    }
    return 0;
}
