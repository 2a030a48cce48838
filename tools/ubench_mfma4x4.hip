// v_mfma_f64_4x4x4f64 on gfx950: issue rate against v_mfma_f64_16x16x4f64
// (independent accumulators, 4 waves per SIMD) and its operand / result lane
// layout (one wave, coded operands).
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma4x4.hip -o tools/build/ubench_mfma4x4
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_m16(double *out, int iters, double s)
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

template <int NACC>
__global__ __launch_bounds__(256) void k_m4(double *out, int iters, double s)
{
    double acc[NACC];
#pragma unroll
    for (int u = 0; u < NACC; u++) acc[u] = 0.0;
    double a = s * threadIdx.x, b = s + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < NACC; u++)
            acc[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[u], 0, 0, 0);
    }
    double r = 0.0;
#pragma unroll
    for (int u = 0; u < NACC; u++) r += acc[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// layout: A lane l = 1000 + l (as the only nonzero "row" contributions are
// tested one at a time), B lane l = 1 if l == sel else 0
__global__ void k_layout(double *out, int sel_a, int sel_b)
{
    const int l = threadIdx.x;
    const double a = (l == sel_a) ? 1.0 : 0.0;
    const double b = (l == sel_b) ? 1.0 : 0.0;
    out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    hipMalloc(&out, sizeof(double) * 256 * ncu * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000, nwg = ncu * 4;
    for (int kind = 0; kind < 2; kind++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            if (kind == 0)
                k_m16<8><<<nwg, 256>>>(out, iters, 1e-9);
            else
                k_m4<8><<<nwg, 256>>>(out, iters, 1e-9);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double per = ms * 1e6 / ((double)iters * 8);   // ns per instruction per SIMD (4 waves)
            if (rep == 1)
                printf("%s: %.2f ns per instruction per SIMD (4 waves/SIMD, 8 independent acc)\n",
                       kind == 0 ? "mfma_f64_16x16x4" : "mfma_f64_4x4x4  ", per / 4.0 * 4.0 / 4.0);
        }
    }
    // layout: for each (A lane, B lane) pair that produces a nonzero output, print
    // the output lane: C lane = f(A lane, B lane)
    double h[64];
    printf("layout (A lane, B lane) -> C lane with 1.0:\n");
    for (int sa = 0; sa < 64; sa++)
        for (int sb = 0; sb < 64; sb++) {
            k_layout<<<1, 64>>>(out, sa, sb);
            hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
            for (int l = 0; l < 64; l++)
                if (h[l] != 0.0) printf("  A%d B%d -> C%d (%g)\n", sa, sb, l, h[l]);
        }
    return 0;
}
