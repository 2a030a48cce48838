// Diagnostic micro-benchmark (not part of the library): stage cycle stamps
// of the 64x64 diagonal factor + inverse -- the library's block_potrf_inv and
// the round-4 variant that carries the panel rows and the inverse's columns
// on wave_factor16x chains (reverted: 29k vs 31k cycles in total) -- to see
// where the chains' time goes.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include
//   -I bundleadjustmentmatlab_amd/csrc tools/ubench_bpi.hip -o tools/build/ubench_bpi
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

__device__ bool bpi_x_dbg(double *As, double *Li, unsigned long long *ts, bool zero_upper = true)
{
    __shared__ __attribute__((aligned(16))) double Vs[16 * LP];   // V_b: 16 x 16 b
    __shared__ __attribute__((aligned(16))) int bad;
    const int tid = threadIdx.x, w = tid >> 6;
    // one trailing block (i, j) of block column k: A_ij -= L_ik L_jk^T
    auto trail = [&](int i, int j, int k) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16_nt(As, 16 * i, 16 * k, As, 16 * j, 16 * k, acc);
        put16(As, 16 * i, 16 * j, acc, -1.0, true);
    };
    // block c of V_b = -sum_{t=c}^{b-1} L_bt Li_tc
    auto vblk = [&](int b, int c) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int t = c; t < b; t++) acc = mfma16_nn(As, 16 * b, 16 * t, Li, 16 * t, 16 * c, acc);
        put16(Vs, 0, 16 * c, acc, -1.0, false);
    };
    // the six 16x16 blocks above the diagonal of L^-1 (everything else is
    // written below); ordered before their readers by the stage barriers
    for (int q = tid; q < 6 * 256; q += blockDim.x) {
        const int b = q >> 8, e = q & 255;
        const int bi = b < 3 ? 0 : (b < 5 ? 1 : 2), bj = b < 3 ? b + 1 : (b < 5 ? b - 1 : 3);
        Li[(16 * bi + (e >> 4)) * LP + 16 * bj + (e & 15)] = 0.0;
    }
#pragma unroll 1
    for (int b = 0; b < 4; b++) {
        const int o = 16 * b, na = 48 - o;   // A rows below the block
        if (w == 0) {
            vseg lo, hi;
            double *ar = As + (o + 16) * LP + o;   // A rows below, block column b
            if (b == 0) {
                lo = vseg{ar, ar, LP, 1, LP, 1, 16};
                hi = vseg{ar + 16 * LP, ar + 16 * LP, LP, 1, LP, 1, 32};
            } else if (b == 1) {
                lo = vseg{Vs, Li + o * LP, 1, LP, 1, LP, 16};
                hi = vseg{ar, ar, LP, 1, LP, 1, 32};
            } else if (b == 2) {
                lo = vseg{ar, ar, LP, 1, LP, 1, 16};
                hi = vseg{Vs, Li + o * LP, 1, LP, 1, LP, 32};
            } else {
                lo = vseg{Vs, Li + o * LP, 1, LP, 1, LP, 16};
                hi = vseg{Vs + 16, Li + o * LP + 16, 1, LP, 1, LP, 32};
            }
            (void)na;
            const bool ok = wave_factor16x(As, Li, o, lo, hi);
            if (tid == 0) bad = (b > 0 ? bad : 0) | (ok ? 0 : 1);
        } else if (b == 1) {   // column 0's trailing blocks right of column 1
            if (w == 1) trail(2, 2, 0);
            else if (w == 2) trail(3, 2, 0);
            else trail(3, 3, 0);
        } else if (b == 2) {   // column 1's
            if (w == 1) trail(3, 3, 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) ts[2 * b] = stamp();
        if (b < 3) {
            // column b+1 of the trailing blocks, and V_b+1: one task per wave
            const int nt = 3 - b;   // blocks (b+1 .. 3, b+1)
            if (w < nt)
                trail(b + 1 + w, b + 1, b);
            else
                vblk(b + 1, w - nt);
            __syncthreads();
            if (threadIdx.x == 0) ts[2 * b + 1] = stamp();
        }
    }
    if (zero_upper) {
        for (int q = tid; q < NB * NB; q += blockDim.x) {   // zero the upper triangle of L
            const int r = q >> 6, c = q & 63;
            if (c > r) As[r * LP + c] = 0.0;
        }
        __syncthreads();
    }
    return bad == 0;
}


__global__ __launch_bounds__(256) void k_bpi(const double *src, unsigned long long *out, int reps)
{
    __shared__ __attribute__((aligned(16))) double As[NB * LP], Li[NB * LP];
    __shared__ unsigned long long ts[16];
    const int tid = threadIdx.x;
    for (int rep = 0; rep < reps; rep++) {
        for (int q = tid; q < NB * NB; q += 256) As[(q >> 6) * LP + (q & 63)] = src[q];
        __syncthreads();
        if (tid == 0) ts[8] = stamp();
        __syncthreads();
        block_potrf_inv(As, Li);
        __syncthreads();
        if (tid == 0) ts[9] = stamp();
        for (int q = tid; q < NB * NB; q += 256) As[(q >> 6) * LP + (q & 63)] = src[q];
        __syncthreads();
        if (tid == 0) ts[10] = stamp();
        __syncthreads();
        bpi_x_dbg(As, Li, ts);
        __syncthreads();
        if (tid == 0) ts[11] = stamp();
        if (tid == 0)
            for (int i = 0; i < 12; i++) out[rep * 12 + i] = ts[i];
        __syncthreads();
    }
}

int main()
{
    const int reps = 32;
    std::vector<double> M(64 * 64), A(64 * 64);
    srand(5);
    for (auto &v : M) v = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < 64; i++)
        for (int j = 0; j < 64; j++) {
            double s = i == j ? 64.0 : 0.0;
            for (int k = 0; k < 64; k++) s += M[i * 64 + k] * M[j * 64 + k];
            A[i * 64 + j] = s;
        }
    double *d;
    unsigned long long *o;
    hipMalloc(&d, sizeof(double) * A.size());
    hipMalloc(&o, sizeof(unsigned long long) * reps * 12);
    hipMemcpy(d, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    for (int it = 0; it < 2; it++) {
        hipLaunchKernelGGL(k_bpi, dim3(1), dim3(256), 0, 0, d, o, reps);
        hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(reps * 12);
    hipMemcpy(h.data(), o, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    auto med = [&](int a, int b) {
        std::vector<double> v;
        for (int r = 1; r < reps; r++) v.push_back((double)(h[r * 12 + b] - h[r * 12 + a]));
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    printf("library block_potrf_inv: %8.0f cycles\n", med(8, 9));
    printf("lane variant whole:      %8.0f cycles\n", med(10, 11));
    printf("  chain 0 %6.0f | M0 %5.0f | chain 1 %6.0f | M1 %5.0f | chain 2 %6.0f | M2 %5.0f | chain 3 %6.0f | tail %5.0f\n",
           med(10, 0), med(0, 1), med(1, 2), med(2, 3), med(3, 4), med(4, 5), med(5, 6), med(6, 11));
    return 0;
}
