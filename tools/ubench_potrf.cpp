// Diagnostic: rocSOLVER dpotrf + dpotrs time on a dense SPD n x n fp64 matrix
// (the reduced camera system of a wide-band scene; not part of the library).
// Build: hipcc -O2 tools/ubench_potrf.cpp -lrocsolver -lrocblas -o tools/build/ubench_potrf
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spd(double *A, int n)
{
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (long long)n * n) return;
    const int r = (int)(q % n), c = (int)(q / n);
    const unsigned h = (unsigned)(r < c ? r * 7919 + c * 104729 : c * 7919 + r * 104729);
    A[q] = (r == c) ? 4.0 * n : ((h % 1000) / 1000.0 - 0.5);
}

int main(int argc, char **argv)
{
    rocblas_handle hd;
    rocblas_create_handle(&hd);
    for (int a = 1; a < argc; a++) {
        const int n = std::atoi(argv[a]);
        double *A, *B;
        rocblas_int *info;
        hipMalloc(&A, sizeof(double) * (size_t)n * n);
        hipMalloc(&B, sizeof(double) * n);
        hipMalloc(&info, sizeof(rocblas_int));
        hipMemset(B, 0, sizeof(double) * n);
        hipEvent_t e0, e1, e2;
        hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
        for (int rep = 0; rep < 4; rep++) {
            k_spd<<<(unsigned)(((long long)n * n + 255) / 256), 256>>>(A, n);
            hipEventRecord(e0, 0);
            rocsolver_dpotrf(hd, rocblas_fill_lower, n, A, n, info);
            hipEventRecord(e1, 0);
            rocsolver_dpotrs(hd, rocblas_fill_lower, n, 1, A, n, B, n);
            hipEventRecord(e2, 0);
            hipEventSynchronize(e2);
            float t1, t2;
            hipEventElapsedTime(&t1, e0, e1);
            hipEventElapsedTime(&t2, e1, e2);
            std::printf("n=%d potrf %.3f ms (%.1f TF/s)  potrs %.3f ms\n", n, t1,
                        (double)n * n * n / 3.0 / (t1 * 1e-3) / 1e12, t2);
        }
        hipFree(A); hipFree(B); hipFree(info);
    }
    return 0;
}
