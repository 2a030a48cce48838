// fp64 MFMA / VALU issue microbenchmark (gfx950): cycles per
// v_mfma_f64_16x16x4f64 with independent accumulators (throughput) and with one
// dependent chain (latency), at 1..4 waves per SIMD; v_fma_f64 for reference.
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma64.hip -o tools/build/ubench_mfma64
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double *out, int iters, double s)
{
    d4 acc[NACC];
#pragma unroll
    for (int u = 0; u < NACC; u++) acc[u] = d4{0.0, 0.0, 0.0, 0.0};
    double a = s * threadIdx.x, b = s + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < NACC; u++)
            acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
    }
    double r = 0.0;
#pragma unroll
    for (int u = 0; u < NACC; u++) r += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_fma(double *out, int iters, double s)
{
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; u++) x[u] = s * (threadIdx.x + u);
    const double a = 1.0000001, b = 1e-9;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = fma(x[u], a, b);
    }
    double r = 0.0;
#pragma unroll
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    double *out;
    hipMalloc(&out, sizeof(double) * 256 * ncu * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    printf("CUs %d, clock %.2f GHz\n", ncu, clk / 1e6);
    for (int wps = 1; wps <= 4; wps++) {   // waves per SIMD = workgroups (4 waves) per CU
        const int nwg = ncu * wps;
        for (int kind = 0; kind < 3; kind++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) k_mfma<8><<<nwg, 256>>>(out, iters, 1e-3);
                if (kind == 1) k_mfma<1><<<nwg, 256>>>(out, iters * 8, 1e-3);
                if (kind == 2) k_fma<<<nwg, 256>>>(out, iters, 1e-3);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double per_simd = (double)iters * 8 * wps;   // instructions per SIMD
            const double ns = ms * 1e6 / per_simd;
            const char *nm[3] = {"mfma f64 16x16x4, 8 indep acc", "mfma f64 16x16x4, 1 chain",
                                 "v_fma_f64, 8 indep"};
            printf("waves/SIMD %d  %-32s %7.3f ms  %.3f ns/instr/SIMD = %.1f cycles @%.2fGHz\n",
                   wps, nm[kind], ms, ns, ns * clk / 1e6, clk / 1e6);
        }
    }
    return 0;
}
