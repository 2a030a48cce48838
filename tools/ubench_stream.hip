// HBM bandwidth microbenchmark (gfx950): the achievable rate of the traffic
// mixes the fused update + linearisation moves (k_update_linearize: ~0.6 GB
// read, ~0.54 GB written per launch at config 3), so its roofline.frac can be
// read against what the chip sustains, not only against the 8 TB/s peak.
//   read      sum of a 1.2 GB array (16-byte loads)
//   write     fill of a 1.2 GB array (16-byte non-temporal stores)
//   copy      0.6 GB read + 0.6 GB written (16-byte loads, plain stores)
//   copy_nt   the same with non-temporal loads and stores (the W stream's policy)
// Each: grid-stride loop, 256 threads, 8 workgroups per CU; 20 launches after
// 5 warmups, hipEvent timing, bytes moved / average time.
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_stream.hip -o tools/build/ubench_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const v2d *__restrict__ a, size_t n, double *out)
{
    v2d s = {0.0, 0.0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s.x == 1.2345e300) out[0] = s.y;   // keep the loads
}

__global__ __launch_bounds__(256) void k_write(v2d *__restrict__ a, size_t n, double v)
{
    const v2d x = {v, v};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(x, a + i);
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const v2d *__restrict__ a, v2d *__restrict__ b,
                                              size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        if (NT) {
            const v2d x = __builtin_nontemporal_load(a + i);
            __builtin_nontemporal_store(x, b + i);
        } else {
            b[i] = a[i];
        }
    }
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

int main()
{
    const size_t bytes = (size_t)1200 << 20;   // 1.2 GiB per array
    const size_t n = bytes / sizeof(v2d);
    v2d *a, *b;
    double *out;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = 8 * ncu;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, double moved, auto launch) {
        for (int k = 0; k < 5; k++) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 20; k++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / 20;
        std::printf("%-8s %8.1f us  %7.1f GB/s  (%.3f GB moved per launch)\n", name, us,
                    moved / (us * 1e-6) / 1e9, moved / 1e9);
    };
    run("read", (double)bytes, [&] { k_read<<<grid, 256>>>(a, n, out); });
    run("write", (double)bytes, [&] { k_write<<<grid, 256>>>(b, n, 1.0); });
    run("copy", (double)bytes, [&] { k_copy<false><<<grid, 256>>>(a, b, n / 2); });
    run("copy_nt", (double)bytes, [&] { k_copy<true><<<grid, 256>>>(a, b, n / 2); });
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(out));
    return 0;
}
