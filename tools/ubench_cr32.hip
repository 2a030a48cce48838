// Diagnostic micro-benchmark (not part of the library): in-kernel cycle
// stamps (s_memtime) of the stages of one cyclic-reduction level record on a
// 32-row tile (cr32_level_body's roles 1 / 2): the neighbour update of D_k
// and the fill, potrf32_inv's four stages, the panel.  One workgroup, the
// tiles already in LDS; median over repetitions.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include
//   tools/ubench_cr32.hip -o tools/build/ubench_cr32
#include "../bundleadjustmentmatlab_amd/csrc/ba_chol.hip"

void kt_begin(ba_ktimer *, hipStream_t) {}
void kt_end(ba_ktimer *, hipStream_t, int) {}
void *ba_dmalloc(size_t bytes)
{
    void *p = nullptr;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}
void ba_dfree(void *p) { (void)hipFree(p); }
int ba_ensure_dyn_lds(const void *, size_t) { return 0; }

#include <algorithm>
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

#define MARK(i)                                   \
    do {                                          \
        __syncthreads();                          \
        if (threadIdx.x == 0) ts[i] = stamp();    \
    } while (0)

#define NST 12

// src: 5 row-major 32 x 32 tiles (D SPD, Lm, Lp, Lq, spare)
__global__ __launch_bounds__(256) void k_cr32_dbg(const double *src, double *dst,
                                                  unsigned long long *out, int reps)
{
    extern __shared__ double pad[];
    if (threadIdx.x == 1000) pad[0] = 0.0;
    out += (size_t)blockIdx.x * reps * (NST + 2);
    __shared__ __attribute__((aligned(16))) double As[T32 * LP], Bs[T32 * LP], Cs[T32 * LP],
        Ds[T32 * LP], Es[T32 * LP];
    __shared__ __attribute__((aligned(16))) double Xs[16 * LP];
    __shared__ unsigned long long ts[NST], rt[2];
    __shared__ int bad32;
    const int tid = threadIdx.x, w = tid >> 6;
    for (int rep = 0; rep < reps; rep++) {
        load_rm32(src, As);
        load_rm32(src + 1024, Bs);
        load_rm32(src + 2048, Cs);
        load_rm32(src + 3072, Ds);
        MARK(0);
        if (tid == 0) rt[0] = __builtin_amdgcn_s_memrealtime();
        {   // fill (role 1): Es = -Ds Bs^T
            d4 f = {0.0, 0.0, 0.0, 0.0};
            f = mfma32_nt(Ds, Bs, f);
            put32(Es, f, -1.0, false);
        }
        MARK(1);
        {   // D_k -= Lm Lm^T + Lp Lp^T (scaled small so D stays SPD)
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma32_nt(Bs, Bs, acc);
            acc = mfma32_nt(Cs, Cs, acc);
            put32(As, acc, -1.0, true);
        }
        MARK(2);
        // potrf32_inv, staged
        Bs[(tid >> 4) * LP + 16 + (tid & 15)] = 0.0;
        if (tid == 0) bad32 = 0;
        if (w == 0 && !wave_factor16(As, Bs, 0) && tid == 0) bad32 = 1;
        MARK(3);
        if (w == 1) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma16_nt(As, 16, 0, Bs, 0, 0, acc);
            put16(As, 16, 0, acc, 1.0, false);
        }
        MARK(4);
        if (w == 0) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma16_nt(As, 16, 0, As, 16, 0, acc);
            put16(As, 16, 16, acc, -1.0, true);
        }
        MARK(5);
        if (w == 0 && !wave_factor16(As, Bs, 16) && tid == 0) bad32 = 1;
        MARK(6);
        if (w == 1) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma16_nn(As, 16, 0, Bs, 0, 0, acc);
            put16(Xs, 0, 0, acc, 1.0, false);
            d4 acc2 = {0.0, 0.0, 0.0, 0.0};
            acc2 = mfma16_nn(Bs, 16, 16, Xs, 0, 0, acc2);
            put16(Bs, 16, 0, acc2, -1.0, false);
        }
        MARK(7);
        {   // panel C L^-T
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            acc = mfma32_nt(Es, Bs, acc);
            __syncthreads();
            put32(Es, acc, 1.0, false);
        }
        MARK(8);
        // the library factor (cr32_chol, L^-1 only) whole, on a fresh copy
        load_rm32(src, As);
        MARK(9);
        cr32_chol(As, Bs, nullptr, Xs, nullptr, nullptr, [](int) {});
        MARK(10);
        store_rm32(dst, Es);
        store_rm32(dst + 1024, Bs);
        MARK(11);
        if (tid == 0) {
            rt[1] = __builtin_amdgcn_s_memrealtime();
            for (int i = 0; i < NST; i++) out[rep * (NST + 2) + i] = ts[i];
            out[rep * (NST + 2) + NST] = rt[0];
            out[rep * (NST + 2) + NST + 1] = rt[1];
        }
    }
}

__global__ __launch_bounds__(256) void k_f16x_dbg(const double *src, unsigned long long *out,
                                                  int reps)
{
    extern __shared__ double pad[];
    if (threadIdx.x == 1000) pad[0] = 0.0;
    out += (size_t)blockIdx.x * reps * 8;
    __shared__ __attribute__((aligned(16))) double As[T32 * LP], Li[T32 * LP], Cm[T32 * LP];
    __shared__ __attribute__((aligned(16))) double Xs[16 * LP];
    __shared__ unsigned long long ts[8];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int rep = 0; rep < reps; rep++) {
        load_rm32(src, As);
        load_rm32(src + 4096, Cm);
        MARK(0);
        if (w == 0) wave_factor16(As, Li, 0);
        MARK(1);
        load_rm32(src, As);
        load_rm32(src + 4096, Cm);
        MARK(2);
        if (w == 0)
            wave_factor16x(As, Li, 0, vseg{As + 16 * LP, As + 16 * LP, LP, 1, LP, 1, 16},
                           vseg{Cm, Cm, LP, 1, LP, 1, 32});
        MARK(3);
        load_rm32(src, As);
        load_rm32(src + 4096, Cm);
        MARK(4);
        cr32_chol(As, Li, Cm, Xs, nullptr, nullptr, [](int) {});
        MARK(5);
        load_rm32(src, As);
        MARK(6);
        cr32_chol(As, nullptr, Cm, Xs, nullptr, nullptr, [](int) {});
        MARK(7);
        if (tid == 0)
            for (int i = 0; i < 8; i++) out[rep * 8 + i] = ts[i];
    }
}

int main(int argc, char **argv)
{
    const int reps = 64;
    const int grid = argc > 1 ? atoi(argv[1]) : 1;
    const size_t padb = argc > 2 ? (size_t)atoi(argv[2]) : 0;
    if (padb) {
        hipFuncSetAttribute((const void *)k_cr32_dbg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)padb);
        hipFuncSetAttribute((const void *)k_f16x_dbg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)padb);
    }
    printf("grid %d, extra LDS %zu B\n", grid, padb);
    std::vector<double> h(5 * 1024, 0.0);  // [4096..]: a panel block C
    srand(7);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    // D = M M^T + 32 I (SPD), neighbours small
    std::vector<double> M(1024);
    for (auto &v : M) v = rnd();
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            double s = (i == j) ? 32.0 : 0.0;
            for (int k = 0; k < 32; k++) s += M[i * 32 + k] * M[j * 32 + k];
            h[i * 32 + j] = s;
        }
    for (int t = 1; t < 4; t++)
        for (int q = 0; q < 1024; q++) h[t * 1024 + q] = 0.1 * rnd();
    double *ds, *dd;
    unsigned long long *dout;
    hipMalloc(&ds, sizeof(double) * h.size());
    hipMalloc(&dd, sizeof(double) * 4096);
    hipMalloc(&dout, sizeof(unsigned long long) * reps * (NST + 2) * grid);
    hipMemcpy(ds, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
    for (int it = 0; it < 3; it++) {
        hipLaunchKernelGGL(k_cr32_dbg, dim3(grid), dim3(256), padb, 0, ds, dd, dout, reps);
        hipDeviceSynchronize();
    }
    std::vector<unsigned long long> o(reps * (NST + 2));
    hipMemcpy(o.data(), dout, sizeof(unsigned long long) * o.size(), hipMemcpyDeviceToHost);
    const char *name[NST - 1] = {"fill (mfma32 + put)", "D update (2 mfma32 + put)",
                                 "f16 block 0", "L10 panel", "A11 update", "f16 block 1",
                                 "Li10 (2 mfma16 chains)", "panel C L^-T", "reload",
                                 "cr32_chol (Li) whole", "stores"};
    printf("cycles (s_memtime), median of %d reps (first rep dropped)\n", reps - 1);
    for (int i = 0; i < NST - 1; i++) {
        std::vector<double> v;
        for (int r = 1; r < reps; r++) v.push_back((double)(o[r * (NST + 2) + i + 1] - o[r * (NST + 2) + i]));
        std::sort(v.begin(), v.end());
        printf("  %-28s %8.0f   (first rep, cold: %llu)\n", name[i], v[v.size() / 2],
               o[i + 1] - o[i]);
    }
    {   // calibration: s_memtime ticks per microsecond (s_memrealtime: 100 MHz)
        std::vector<double> v;
        for (int r = 1; r < reps; r++) {
            const unsigned long long *q = &o[r * (NST + 2)];
            v.push_back((double)(q[11] - q[0]) / ((double)(q[NST + 1] - q[NST]) / 100.0));
        }
        std::sort(v.begin(), v.end());
        printf("  s_memtime ticks per us: %.1f\n", v[v.size() / 2]);
    }
    {
        unsigned long long *d2;
        hipMalloc(&d2, sizeof(unsigned long long) * reps * 8 * grid);
        for (int it = 0; it < 3; it++) {
            hipLaunchKernelGGL(k_f16x_dbg, dim3(grid), dim3(256), padb, 0, ds, d2, reps);
            hipDeviceSynchronize();
        }
        std::vector<unsigned long long> o2(reps * 8);
        hipMemcpy(o2.data(), d2, sizeof(unsigned long long) * o2.size(), hipMemcpyDeviceToHost);
        const char *nm[4] = {"wave_factor16", "wave_factor16x (F0 shape)", "cr32_chol (Li + panel)",
                             "cr32_chol (panel only)"};
        const int a[4] = {0, 2, 4, 6};
        for (int k = 0; k < 4; k++) {
            std::vector<double> v;
            for (int r = 1; r < reps; r++) v.push_back((double)(o2[r * 8 + a[k] + 1] - o2[r * 8 + a[k]]));
            std::sort(v.begin(), v.end());
            printf("  %-28s %8.0f   (first rep, cold: %llu)\n", nm[k], v[v.size() / 2],
                   o2[a[k] + 1] - o2[a[k]]);
        }
    }
    return 0;
}
