// ba_camera.h -- device view of one camera for the projections of the
// linearisation kernels (ba_kernels.hip) and the batched resection
// (ba_resect.hip): the reference's reproject_point.h:16-57 with the per-camera
// rotations hoisted into a table (vl_rodrigues).
#pragma once
#include "ba_internal.h"
#include "vlg_math.h"

#define H_FD VLG_FD_H

// -------------------------------------------------------------------------
// camera j as the projections see it.  Euclidean (NA = 6 / 7 / 10): a0, the
// calibration of reproject_point.h:26-41 and the hoisted rotations
// R(w), R(w + h e_k), R(w + 0) (k_rotations); projective (NA = BA_PROJ_NA):
// P = a0 (mex_bundle_proj_1_XABeUVWeAeB.c:21-22), K4 / rot unused.
//   project(b, x)         x = proj(a0, b)
//   project_dcam(k, b, x) x = proj(a0 + h e_k, b), a1 formed component-wise
//                         as a0 + h * da (mex_bundle_1 :30-33, proj :47-51)
//   project_col(c, b, x)  column c of [A | B]: c < NA as project_dcam, else
//                         proj(a0, b + h e_{c-NA}) (mex_bundle_1 :59-66)
// -------------------------------------------------------------------------
template <int NA, bool PROJ = (NA == BA_PROJ_NA)>
struct cam_view;

template <int NA>
struct cam_view<NA, false> {
    double a0[NA], k4[4], Kc[9], Rl[9];
    const double *R;
    __device__ __forceinline__ cam_view(const double *__restrict__ a,
                                        const double *__restrict__ K4,
                                        const double *__restrict__ rot, int j)
        : cam_view(a, K4, rot, j, j)
    {
    }
    // jr: the camera's row of rot (a staged copy of part of the table, e.g.
    // in LDS), j: its index into a and K4
    __device__ __forceinline__ cam_view(const double *__restrict__ a,
                                        const double *__restrict__ K4,
                                        const double *__restrict__ rot, int jr, int j)
    {
#pragma unroll
        for (int c = 0; c < NA; c++) a0[c] = a[(size_t)NA * j + c];
#pragma unroll
        for (int c = 0; c < 4; c++) k4[c] = K4[4 * (size_t)j + c];
        R = rot + 45 * (size_t)jr;
#pragma unroll
        for (int q = 0; q < 9; q++) Rl[q] = R[q];
        vlg_calib(Kc, k4, a0, NA - 6);
    }
    __device__ __forceinline__ void project(const double b[3], double x[2]) const
    {
        vlg_project(Kc, Rl, a0 + 3, b, x);
    }
    __device__ __forceinline__ void project_dcam(int k, const double b[3], double x[2]) const
    {
        double a1[NA], Kc1[9], Rk[9];
#pragma unroll
        for (int c = 0; c < NA; c++) a1[c] = a0[c] + H_FD * ((c == k) ? 1.0 : 0.0);
        vlg_calib(Kc1, k4, a1, NA - 6);
        const double *Rs = R + 9 * ((k < 3) ? (1 + k) : 4);
#pragma unroll
        for (int q = 0; q < 9; q++) Rk[q] = Rs[q];
        vlg_project(Kc1, Rk, a1 + 3, b, x);
    }
    // FD column col of [A | B] without a branch: col < NA perturbs camera
    // component col (as project_dcam), col >= NA point component col - NA
    // with the unperturbed camera (mex_bundle_1 :43-70: K, R(w), T of a)
    __device__ __forceinline__ void project_col(int col, const double b[3], double x[2]) const
    {
        const bool cam = col < NA;
        double a1[NA], b1[3], Kc1[9], Rk[9];
#pragma unroll
        for (int c = 0; c < NA; c++)
            a1[c] = cam ? a0[c] + H_FD * ((c == col) ? 1.0 : 0.0) : a0[c];
#pragma unroll
        for (int c = 0; c < 3; c++)
            b1[c] = cam ? b[c] : b[c] + H_FD * ((c == col - NA) ? 1.0 : 0.0);
        vlg_calib(Kc1, k4, a1, NA - 6);
        const double *Rs = R + 9 * ((col < 3) ? (1 + col) : (cam ? 4 : 0));
#pragma unroll
        for (int q = 0; q < 9; q++) Rk[q] = Rs[q];
        vlg_project(Kc1, Rk, a1 + 3, b1, x);
    }
};

template <int NA>
struct cam_view<NA, true> {
    double a0[NA];
    __device__ __forceinline__ cam_view(const double *__restrict__ a, const double *, const double *,
                                        int j)
    {
#pragma unroll
        for (int c = 0; c < NA; c++) a0[c] = a[(size_t)NA * j + c];
    }
    __device__ __forceinline__ void project(const double b[3], double x[2]) const
    {
        vlg_project_proj(a0, b, x);
    }
    __device__ __forceinline__ void project_dcam(int k, const double b[3], double x[2]) const
    {
        double a1[NA];
#pragma unroll
        for (int c = 0; c < NA; c++) a1[c] = a0[c] + H_FD * ((c == k) ? 1.0 : 0.0);
        vlg_project_proj(a1, b, x);
    }
    __device__ __forceinline__ void project_col(int col, const double b[3], double x[2]) const
    {
        const bool cam = col < NA;
        double a1[NA], b1[3];
#pragma unroll
        for (int c = 0; c < NA; c++)
            a1[c] = cam ? a0[c] + H_FD * ((c == col) ? 1.0 : 0.0) : a0[c];
#pragma unroll
        for (int c = 0; c < 3; c++)
            b1[c] = cam ? b[c] : b[c] + H_FD * ((c == col - NA) ? 1.0 : 0.0);
        vlg_project_proj(a1, b1, x);
    }
};

// -------------------------------------------------------------------------
// rotations: R(a), R(a + h e_k) k = 0..2, R(a + 0) per camera (5 x 9)
// -------------------------------------------------------------------------
// rotation k of the table alone (k = 0: R(w); k = 1..4: as below)
__device__ __forceinline__ void rotation_k(const double w[3], int k, double *__restrict__ out)
{
    double R[9], w1[3];
#pragma unroll
    for (int c = 0; c < 3; c++) w1[c] = k == 0 ? w[c] : w[c] + H_FD * ((c == k - 1) ? 1.0 : 0.0);
    vlg_rodrigues(R, w1);
#pragma unroll
    for (int q = 0; q < 9; q++) out[9 * k + q] = R[q];
}

__device__ __forceinline__ void rotations5(const double w[3], double *__restrict__ out)
{
    double R[9];
    vlg_rodrigues(R, w);
#pragma unroll
    for (int q = 0; q < 9; q++) out[q] = R[q];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        // derivative_camera (mex_bundle_1_XABeUVWeAeB.c:30-33): a1 = a0 + h*da,
        // da = e_k for k < 3; for k >= 3 the rotation part is a0 + h*0.
        double w1[3];
#pragma unroll
        for (int c = 0; c < 3; c++) w1[c] = w[c] + H_FD * ((c == k) ? 1.0 : 0.0);
        vlg_rodrigues(R, w1);
#pragma unroll
        for (int q = 0; q < 9; q++) out[9 * (1 + k) + q] = R[q];
    }
}

