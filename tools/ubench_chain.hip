// Diagnostic: dependent-chain latency (cycles per operation, one wave) of the
// operations on the Cholesky pivot chain (wave_factor16, ba_chol.hip):
// v_fma_f64, v_mul_f64, v_rsq_f64, the DPP row broadcast of a double, and one
// whole pivot step.  Not part of the library.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/ubench_chain.hip -o tools/build/ubench_chain
#include <hip/hip_runtime.h>
#include <cstdio>

template <int Q> __device__ __forceinline__ double rowbcast_c(double v)
{
    const long long u = __builtin_bit_cast(long long, v);
    const long long r = __builtin_amdgcn_mov_dpp(u, 0x150 + Q, 0xf, 0xf, true);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ unsigned long long clk()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define N 256
__global__ void k_chain(double *out, unsigned long long *cyc, double seed)
{
    double x = seed + threadIdx.x * 1e-3, y = 1.0;
    unsigned long long t0, t1;
    // 0: fma chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = fma(x, 0.999999, 1e-7);
    t1 = clk();
    cyc[0] = t1 - t0;
    // 1: mul chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = x * 1.0000001;
    t1 = clk();
    cyc[1] = t1 - t0;
    // 2: rsq chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = __builtin_amdgcn_rsq(x);
    t1 = clk();
    cyc[2] = t1 - t0;
    // 3: DPP row broadcast + add chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = rowbcast_c<3>(x) + 1e-9;
    t1 = clk();
    cyc[3] = t1 - t0;
    // 4: one pivot step: bcast, fma, bcast, rsq + 2 Newton steps, scale
    t0 = clk();
#pragma unroll 4
    for (int i = 0; i < N / 8; i++) {
        const double b = rowbcast_c<1>(x);
        double d = fma(-x, b, 2.0);
        const double piv = rowbcast_c<1>(d) + 1.5;
        double r = __builtin_amdgcn_rsq(piv);
        const double hp = 0.5 * piv;
        r = r * fma(-hp * r, r, 1.5);
        r = r * fma(-hp * r, r, 1.5);
        x = d * r;
        y += r;
    }
    t1 = clk();
    cyc[4] = t1 - t0;
    // 5: add chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = x + 1e-9;
    t1 = clk();
    cyc[5] = t1 - t0;
    out[threadIdx.x] = x + y;
}

int main()
{
    double *out;
    unsigned long long *cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMallocManaged(&cyc, 8 * sizeof(unsigned long long));
    for (int rep = 0; rep < 3; rep++) {
        k_chain<<<1, 64>>>(out, cyc, 1.5);
        hipDeviceSynchronize();
        // s_memtime counts at the 100 MHz reference clock: x 24 ~ shader cycles at 2.4 GHz
        std::printf("memtime ticks per op (x24 = cycles @2.4GHz): fma %.2f  mul %.2f  rsq %.2f  "
                    "dpp+add %.2f  add %.2f  | pivot step %.2f\n",
                    cyc[0] / 256.0, cyc[1] / 256.0, cyc[2] / 256.0, cyc[3] / 256.0,
                    cyc[5] / 256.0, cyc[4] / 32.0);
    }
    return 0;
}
