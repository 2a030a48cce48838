// Variants of the 16-row pivot-chain factor (ba_chol.hip: wave_factor16x) on
// one wave: cycles (s_memtime) per call and a bit-for-bit comparison of L,
// L^-1 and the substituted vectors against the library's version.
//   V1: per pivot, every broadcast of the column first (distinct registers),
//       then the rank-1 / substitution FMAs -- no FMA waits on the DPP just
//       before it
//   V2: V1 with the broadcasts of columns q >= c + 3 read from LDS (one
//       16-double column store per pivot; LDS reads leave the VALU issue)
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include
//        tools/ubench_f16v.hip -o tools/build/ubench_f16v
#include "../bundleadjustmentmatlab_amd/csrc/ba_chol.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// host helpers of the library that ba_chol.hip's host code references (never
// called here)
void kt_begin(struct ba_ktimer *, hipStream_t) {}
void kt_end(struct ba_ktimer *, hipStream_t, int) {}
void *ba_dmalloc(size_t) { return nullptr; }
int ba_ensure_dyn_lds(const void *, size_t) { return 0; }
void ba_dfree(void *) {}

template <int V>
__device__ __forceinline__ bool wave_factor16v(double *As, double *Li, int o, vseg lo, vseg hi,
                                               double *colx)
{
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
    __builtin_amdgcn_wave_barrier();
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
        if (V == 2 && c + 3 < 16 && lane < 16) colx[16 * c + lane] = d[c];   // column c of L
        double bq[16];
        if (c + 1 < 16) {
            const double b = rowbcast(d[c], c + 1);
            d[c + 1] = fma(-d[c], b, d[c + 1]);
            y = rsq(rowbcast(d[c + 1], c + 1));
            x[c + 1] = fma(-b, x[c], x[c + 1]);
        }
#pragma unroll
        for (int q = c + 2; q < 16; q++) {
            if (V == 2 && q >= c + 3) {
                __builtin_amdgcn_wave_barrier();
                bq[q] = colx[16 * c + q];   // broadcast read (every lane one address)
            } else {
                bq[q] = rowbcast(d[c], q);
            }
        }
#pragma unroll
        for (int q = c + 2; q < 16; q++) {
            d[q] = fma(-d[c], bq[q], d[q]);
            x[q] = fma(-bq[q], x[c], x[q]);
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

// V3: wave 0 runs the pivot chain and the factor's rank-1 updates (every
// 16-lane row a copy of the rows), publishing each column of L and its pivot
// scale in LDS; wave 1 runs the substitutions of all 64 lanes (L^-1 columns in
// lanes 0..15, the vectors in 16..63) from those columns, one pivot behind.
// The same operations on every value in the same order: bit-identical.
__device__ __forceinline__ bool wave_factor16s(double *As, double *Li, int o, vseg lo, vseg hi,
                                               double *colx, volatile int *flag, int *okp)
{
    __shared__ double ident[33];
    const int tid = threadIdx.x, w = tid >> 6;
    const int lane = tid & 63, r = lane & 15;
    if (w == 0) {
        double d[16];
#pragma unroll
        for (int c = 0; c < 16; c++) d[c] = As[(o + r) * LP + o + c];
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
            if (lane < 16) colx[17 * c + lane] = d[c];   // column c of L (rows > c used)
            if (lane == 0) colx[17 * c + 16] = y;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) flag[0] = c + 1;
            if (c + 1 < 16) {
                const double b = rowbcast(d[c], c + 1);
                d[c + 1] = fma(-d[c], b, d[c + 1]);
                y = rsq(rowbcast(d[c + 1], c + 1));
            }
#pragma unroll
            for (int q = c + 2; q < 16; q++) {
                const double b = rowbcast(d[c], q);
                d[q] = fma(-d[c], b, d[q]);
            }
        }
        double dg = 1.0;
#pragma unroll
        for (int c = 0; c < 16; c++)
            if (r == c) dg = d[c];
        const bool ok = __all(lane >= 16 || (dg > 0.0 && dg < __builtin_inf()));
        if (lane < 16) {
#pragma unroll
            for (int c = 0; c < 16; c++) As[(o + r) * LP + o + c] = (c <= r) ? d[c] : 0.0;
        }
        if (lane == 0) *okp = ok ? 1 : 0;
    } else if (w == 1) {
        if (lane < 33) ident[lane] = lane == 16 ? 1.0 : 0.0;
        const bool up = lane >= 32;
        const int idx = up ? lane - 32 : lane - 16;
        const double *sin = up ? hi.in : lo.in;
        const bool act = lane >= 16 && sin != nullptr && idx < (up ? hi.n : lo.n);
        const double *pin =
            act ? sin + idx * (up ? hi.irs : lo.irs) : (lane < 16 ? ident + 16 - r : ident);
        const int ics = act ? (up ? hi.ics : lo.ics) : 1;
        double x[16];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 16; q++) x[q] = pin[q * ics];
#pragma unroll
        for (int c = 0; c < 16; c++) {
            while (flag[0] <= c) __builtin_amdgcn_s_sleep(0);
            __builtin_amdgcn_wave_barrier();
            const double *col = colx + 17 * c;
            x[c] = x[c] * col[16];
#pragma unroll
            for (int q = c + 1; q < 16; q++) x[q] = fma(-col[q], x[c], x[q]);
        }
        if (lane < 16) {
#pragma unroll
            for (int c = 0; c < 16; c++) Li[(o + c) * LP + o + r] = x[c];
        } else if (act) {
            double *po = (up ? hi.out : lo.out) + idx * (up ? hi.ors : lo.ors);
            const int ocs = up ? hi.ocs : lo.ocs;
#pragma unroll
            for (int c = 0; c < 16; c++) po[c * ocs] = x[c];
        }
    }
    __syncthreads();
    return *okp != 0;
}

#define MK(i)                                                                      \
    do {                                                                           \
        __syncthreads();                                                           \
        if (tid == 0) ts[i] = __builtin_amdgcn_s_memtime();                        \
        __syncthreads();                                                           \
    } while (0)

// variant v (0 = library) on the F0 shape; results to res[v][...]
__global__ __launch_bounds__(256) void k_f16v(const double *src, unsigned long long *out,
                                              double *res, int reps)
{
    __shared__ __attribute__((aligned(16))) double As[T32 * LP], Li[T32 * LP], Cm[T32 * LP];
    __shared__ __attribute__((aligned(16))) double colx[17 * 16];
    __shared__ int flag[1], okv[1];
    __shared__ unsigned long long ts[10];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int rep = 0; rep < reps; rep++) {
        for (int v = 0; v < 4; v++) {
            load_rm32(src, As);
            if (tid == 0) flag[0] = 0;
            load_rm32(src + 4096, Cm);
            for (int q = tid; q < T32 * LP; q += 256) Li[q] = 0.0;
            MK(2 * v);
            const vseg lo{As + 16 * LP, As + 16 * LP, LP, 1, LP, 1, 16};
            const vseg hi{Cm, Cm, LP, 1, LP, 1, 32};
            if (v == 3) {
                wave_factor16s(As, Li, 0, lo, hi, colx, flag, okv);
            } else if (w == 0) {
                if (v == 0) wave_factor16x(As, Li, 0, lo, hi);
                else if (v == 1) wave_factor16v<1>(As, Li, 0, lo, hi, colx);
                else wave_factor16v<2>(As, Li, 0, lo, hi, colx);
            }
            MK(2 * v + 1);
            if (rep == 0) {
                double *rv = res + (size_t)v * 3 * T32 * LP;
                for (int q = tid; q < T32 * LP; q += 256) {
                    rv[q] = As[q];
                    rv[T32 * LP + q] = Li[q];
                    rv[2 * T32 * LP + q] = Cm[q];
                }
            }
        }
        if (tid == 0)
            for (int i = 0; i < 8; i++) out[rep * 8 + i] = ts[i];
    }
}

int main()
{
    const int reps = 64;
    std::vector<double> h(5 * 1024, 0.0);
    srand(7);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
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
    double *ds, *dres;
    unsigned long long *dout;
    const size_t nres = 4 * 3 * (size_t)T32 * LP;
    hipMalloc(&ds, sizeof(double) * h.size());
    hipMalloc(&dres, sizeof(double) * nres);
    hipMalloc(&dout, sizeof(unsigned long long) * reps * 8);
    hipMemcpy(ds, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
    for (int it = 0; it < 3; it++) {
        hipLaunchKernelGGL(k_f16v, dim3(1), dim3(256), 0, 0, ds, dout, dres, reps);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 1;
        }
    }
    std::vector<unsigned long long> o(reps * 8);
    std::vector<double> r(nres);
    hipMemcpy(o.data(), dout, sizeof(unsigned long long) * o.size(), hipMemcpyDeviceToHost);
    hipMemcpy(r.data(), dres, sizeof(double) * nres, hipMemcpyDeviceToHost);
    const char *nm[4] = {"wave_factor16x (library)", "V1 broadcasts first", "V2 + LDS columns", "V3 two waves"};
    const size_t per = 3 * (size_t)T32 * LP;
    for (int v = 0; v < 4; v++) {
        std::vector<double> t;
        for (int k = 1; k < reps; k++) t.push_back((double)(o[k * 8 + 2 * v + 1] - o[k * 8 + 2 * v]));
        std::sort(t.begin(), t.end());
        size_t diff = 0;
        for (size_t q = 0; q < per; q++)
            if (memcmp(&r[q], &r[v * per + q], sizeof(double)) != 0) diff++;
        printf("  %-28s %8.0f cycles   differing doubles vs library: %zu\n", nm[v],
               t[t.size() / 2], diff);
    }
    return 0;
}
