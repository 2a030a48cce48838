// Diagnostic micro-benchmark (not part of the library): in-kernel cycle
// stamps of the phases of block_potrf_inv and k_cr_factor on one SPD tile.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include
//   tools/ubench_crf.hip -o tools/ubench_crf
#include "../bundleadjustmentmatlab_amd/csrc/ba_chol.hip"

void kt_begin(ba_ktimer *, hipStream_t) {}
void kt_end(ba_ktimer *, hipStream_t, int) {}
// the library's caching allocator (ba_solver.cpp) is not linked here either
void *ba_dmalloc(size_t bytes)
{
    void *p = nullptr;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}
void ba_dfree(void *p) { (void)hipFree(p); }

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

#define MARK(i) do { __syncthreads(); if (threadIdx.x == 0) ts[i] = stamp(); } while (0)

__device__ void bpi_dbg(double *As, double *Li, unsigned long long *ts)
{
    __shared__ double Xs[4][16 * LP];
    __shared__ __attribute__((aligned(16))) int bad;
    const int tid = threadIdx.x, w = tid >> 6;
    for (int q = tid; q < NB * LP; q += blockDim.x) Li[q] = 0.0;
    if (tid == 0) bad = 0;
    MARK(1);
    for (int kb = 0; kb < 4; kb++) {
        const int o = 16 * kb;
        if (w == 0 && !wave_factor16(As, Li, o) && (tid & 63) == 0) bad = 1;
        MARK(2 + 3 * kb);
        if (w >= 1 && kb + w <= 3) {
            const int i = kb + w;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma16_nt(As, 16 * i, o, Li, o, o, acc);
            put16(As, 16 * i, o, acc, 1.0, false);
        }
        MARK(3 + 3 * kb);
        int pidx = 0;
        for (int j = kb + 1; j < 4; j++)
            for (int i = j; i < 4; i++, pidx++)
                if ((pidx & 3) == w) {
                    d4 acc = {0.0, 0.0, 0.0, 0.0};
                    acc = mfma16_nt(As, 16 * i, o, As, 16 * j, o, acc);
                    put16(As, 16 * i, 16 * j, acc, -1.0, true);
                }
        MARK(4 + 3 * kb);
    }
    for (int i = 1; i < 4; i++) {
        if (w < i) {
            const int j = w;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int t = j; t < i; t++) acc = mfma16_nn(As, 16 * i, 16 * t, Li, 16 * t, 16 * j, acc);
            put16(Xs[w], 0, 0, acc, 1.0, false);
            d4 acc2 = {0.0, 0.0, 0.0, 0.0};
            acc2 = mfma16_nn(Li, 16 * i, 16 * i, Xs[w], 0, 0, acc2);
            put16(Li, 16 * i, 16 * j, acc2, -1.0, false);
        }
        MARK(13 + i);
    }
    for (int q = tid; q < NB * NB; q += blockDim.x) {
        const int r = q >> 6, c = q & 63;
        if (c > r) As[r * LP + c] = 0.0;
    }
    MARK(17);
}

__global__ __launch_bounds__(256) void k_crf_dbg(double *S, long long lds, double *linv,
                                                 double *crL, const double *rhs, double *y,
                                                 unsigned long long *out)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP, *Cs = sm + 2 * NB * LP;
    __shared__ double rk[NB];
    __shared__ double part[4][NB];
    __shared__ unsigned long long ts[32];
    const int tid = threadIdx.x;
    const int e = 1, p = 0, q = 2, nt = 3;
    MARK(0);
    load_tile(S, lds, e, e, As);
    if (tid < NB) rk[tid] = rhs[(long long)NB * e + tid];
    MARK(18);
    bpi_dbg(As, Bs, ts);
    gemv64(Bs, rk, part, y + (long long)NB * e, 1.0);
    MARK(19);
    store_rowmajor(linv + (long long)NB * NB * e, Bs);
    MARK(20);
    d4 acc[2][2];
    load_tile_t(S, lds, e, p, Cs);
    MARK(21);
    mfma_64x64(Cs, Bs, acc);
    MARK(22);
    acc_to_lds(acc, Cs, 1.0, false);
    MARK(23);
    store_rowmajor(crL + (long long)NB * NB * e, Cs);
    MARK(24);
    load_tile(S, lds, q, e, Cs);
    __syncthreads();
    mfma_64x64(Cs, Bs, acc);
    __syncthreads();
    acc_to_lds(acc, Cs, 1.0, false);
    __syncthreads();
    store_rowmajor(crL + (long long)NB * NB * (nt + e), Cs);
    MARK(25);
    if (tid == 0)
        for (int i = 0; i < 26; i++) out[i] = ts[i];
}


// current wave_factor16 with stamps: [0] LDS read, [1] pivot loop, [2] L write, [3] inverse, [4] Li write
__device__ void wf16_dbg(double *As, double *Bs, int o, unsigned long long *tw)
{
    const int r = threadIdx.x & 63;
    double d[16], rd[16];
    unsigned long long t0 = stamp();
#pragma unroll
    for (int c = 0; c < 16; c++) d[c] = (r < 16) ? As[(o + r) * LP + o + c] : 0.0;
    asm volatile("" ::"v"(d[0]), "v"(d[15]));
    __builtin_amdgcn_s_waitcnt(0xc07f);
    unsigned long long t1 = stamp();
    auto rsq = [&](double piv) {
        if (!(piv > 0.0)) piv = 1.0;
        double y = __builtin_amdgcn_rsq(piv);
        const double hp = 0.5 * piv;
        y = y * fma(-hp * y, y, 1.5);
        y = y * fma(-hp * y, y, 1.5);
        return y;
    };
    double pv = rdlane(d[0], 0);
    double y = rsq(pv);
#pragma unroll
    for (int c = 0; c < 16; c++) {
        rd[c] = y;
        d[c] = (r == c) ? pv * y : ((r > c) ? d[c] * y : 0.0);
        if (c + 1 < 16) {
            d[c + 1] = fma(-d[c], rowbcast(d[c], c + 1), d[c + 1]);
            pv = rdlane(d[c + 1], c + 1);
            y = rsq(pv);
        }
#pragma unroll
        for (int q = c + 2; q < 16; q++) d[q] = fma(-d[c], rowbcast(d[c], q), d[q]);
    }
    asm volatile("" ::"v"(d[15]), "v"(d[0]), "v"(d[7]));
    unsigned long long t2 = stamp();
    if (r < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) As[(o + r) * LP + o + c] = (c <= r) ? d[c] : 0.0;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    unsigned long long t3 = stamp();
    double x[16];
#pragma unroll
    for (int q = 0; q < 16; q++) x[q] = (q == r) ? 1.0 : 0.0;
#pragma unroll
    for (int t = 0; t < 16; t++) {
        x[t] = x[t] * rd[t];
#pragma unroll
        for (int q = t + 1; q < 16; q++) x[q] = fma(-rowbcast(d[t], q), x[t], x[q]);
    }
    asm volatile("" ::"v"(x[15]), "v"(x[0]));
    unsigned long long t4 = stamp();
    if (r < 16) {
#pragma unroll
        for (int c = 0; c < 16; c++) Bs[(o + c) * LP + o + r] = x[c];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    unsigned long long t5 = stamp();
    tw[0] = t1 - t0; tw[1] = t2 - t1; tw[2] = t3 - t2; tw[3] = t4 - t3; tw[4] = t5 - t4;
}

__global__ __launch_bounds__(256) void k_wf_dbg(const double *S, long long lds, unsigned long long *out)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    load_tile(S, lds, 0, 0, As);
    __syncthreads();
    unsigned long long tw[5];
    if (threadIdx.x < 64) wf16_dbg(As, Bs, 0, tw);
    if (threadIdx.x == 0)
        for (int q = 0; q < 5; q++) out[q] = tw[q];
}

// the library's block_potrf_inv, timed whole
__global__ __launch_bounds__(256) void k_bpi_lib(const double *S, long long lds,
                                                 unsigned long long *out)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *As = sm, *Bs = sm + NB * LP;
    __shared__ unsigned long long ts[2];
    load_tile(S, lds, 1, 1, As);
    __syncthreads();
    if (threadIdx.x == 0) ts[0] = stamp();
    block_potrf_inv(As, Bs, false);
    if (threadIdx.x == 0) out[0] = stamp() - ts[0];
}

int main()
{
    const int n = 192;
    std::vector<double> M((size_t)n * n), h((size_t)n * n);
    srand(1);
    for (auto &v : M) v = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double s = (i == j) ? n : 0.0;
            for (int k = 0; k < n; k++) s += M[i * n + k] * M[j * n + k];
            h[i + (size_t)n * j] = s;
        }
    double *S, *linv, *crL, *rhs, *y;
    unsigned long long *out;
    hipMalloc(&S, sizeof(double) * n * n);
    hipMalloc(&linv, sizeof(double) * 3 * 64 * 64);
    hipMalloc(&crL, sizeof(double) * 6 * 64 * 64);
    hipMalloc(&rhs, sizeof(double) * n);
    hipMalloc(&y, sizeof(double) * n);
    hipMalloc(&out, sizeof(unsigned long long) * 32);
    hipMemcpy(S, h.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    hipMemset(rhs, 0, sizeof(double) * n);
    const size_t smem3 = sizeof(double) * 3 * NB * LP;
    hipFuncSetAttribute((const void *)k_crf_dbg, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    unsigned long long ho[32];
    for (int it = 0; it < 3; it++) {
        k_crf_dbg<<<1, 256, smem3>>>(S, n, linv, crL, rhs, y, out);
        hipMemcpy(ho, out, sizeof(unsigned long long) * 26, hipMemcpyDeviceToHost);
    }
    const char *nm[26] = {"start", "zeroLi", "f16_0", "pan_0", "trail_0", "f16_1", "pan_1",
                          "trail_1", "f16_2", "pan_2", "trail_2", "f16_3", "pan_3", "trail_3",
                          "inv_1", "inv_2", "inv_3", "zeroU", "load", "gemv", "store_linv",
                          "load_t", "mfma", "acc_lds", "store_crL", "panel_q"};
    const int order[26] = {0, 18, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17,
                           19, 20, 21, 22, 23, 24, 25};
    for (int k = 1; k < 26; k++)
        printf("%-11s %8llu\n", nm[order[k]], ho[order[k]] - ho[order[k - 1]]);
    printf("total      %8llu cycles\n", ho[25] - ho[0]);
    hipFuncSetAttribute((const void *)k_wf_dbg, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    for (int it = 0; it < 3; it++) {
        k_wf_dbg<<<1, 256, smem3>>>(S, n, out);
        hipMemcpy(ho, out, sizeof(unsigned long long) * 5, hipMemcpyDeviceToHost);
    }
    hipFuncSetAttribute((const void *)k_bpi_lib, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem3);
    for (int it = 0; it < 3; it++) {
        k_bpi_lib<<<1, 256, smem3>>>(S, n, out);
        hipMemcpy(ho + 8, out, sizeof(unsigned long long), hipMemcpyDeviceToHost);
    }
    printf("library block_potrf_inv: %llu cycles\n", ho[8]);
    printf("wave_factor16: lds read %llu  pivot loop %llu  L write %llu  inverse %llu  Li write %llu\n",
           ho[0], ho[1], ho[2], ho[3], ho[4]);
    return 0;
}
