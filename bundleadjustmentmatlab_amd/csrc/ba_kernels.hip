// ba_kernels.hip -- gfx950 kernels of one LM iteration (fp64), Euclidean
// (NA = 6 / 7 / 10) and projective (NA = BA_PROJ_NA = 12: the camera is P(:),
// mex_bundle_proj_{1,3}*.c -- the same loops with reproject_projective_point).
//
// Reference path (toolbox/bundle/):
//   k_rotations        vl_rodrigues per camera, hoisted out of reproject_point.h:44
//   k_linearize        mex_bundle_1_XABeUVWeAeB.c:192-256 (projection + FD Jacobians)
//                      and the per-point half of :266-334 (W_ij, V_i, eB_i)
//   k_camera_reduce    the per-camera half of :266-334 (U_j, eA_j)
//   k_damp_point       bundle_euclid.m:168-184 (V* = damp(V), pinv, Y = W V*^-1)
//   k_schur            mex_bundle_2_Se_.c:72-155 (S_jk, e_) on the co-visible blocks
//   k_linearize_chunk  fast path: linearisation per chunk of points + U/eA partials
//   k_schur_group      fast path: damp + V*^-1 + Y + S / e_ partials per group of chunks
//   k_assemble         dense S for the reduced solve (bundle_euclid.m:193)
//   k_camera_update    mex_bundle_3_db_new.c:137-140 (a_new) + rotations of a_new
//   k_point_update     mex_bundle_3_db_new.c:99-166 (db, b_new, new projections)
//                      and the cost / rho terms of bundle_euclid.m:205-217
//
// Parity: every per-element expression keeps the reference's operation order,
// the file is compiled with -ffp-contract=off, and every reduction that the
// reference performs sequentially (U_j over points, V_i / eB_i over cameras,
// S_jk / e_j over points) is performed sequentially in the same ascending order
// here, so X_hat, A, B, e, U, V, W, eA, eB, Y, S and e_ are bit-identical to
// the oracle's (and the reference's, modulo libm).  Only the scalar cost sums
// use tree reductions (MATLAB's BLAS dot order is unknowable anyway).
#include "ba_internal.h"
#include "ba_camera.h"
#include "vlg_math.h"
#include "../../include/vlgba.h"

typedef double d4 __attribute__((ext_vector_type(4)));

// Diagnostic build only (make stamps): thread 0 of every workgroup adds the
// s_memtime cycles of each phase of the fast-path kernels to g_stamp.
#ifdef BA_STAMPS
__device__ unsigned long long g_stamp[32];
#define STAMP_DECL unsigned long long st_prev_ = __builtin_amdgcn_s_memtime()
#define STAMP(i)                                                                    \
    do {                                                                            \
        if (threadIdx.x == 0) {                                                     \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
            atomicAdd(&g_stamp[i], t_ - st_prev_);                                  \
            st_prev_ = t_;                                                          \
        }                                                                           \
    } while (0)
extern "C" int vlgba_debug_stamps(unsigned long long *out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(g_stamp)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define STAMP_DECL
#define STAMP(i)
#endif

typedef double v2d __attribute__((ext_vector_type(2)));   // (for the non-temporal builtins)

// -------------------------------------------------------------------------
// block reduction of one double per thread -> partial[blockIdx.x]
// -------------------------------------------------------------------------
template <int BS>
__device__ __forceinline__ void block_sum_to(double v, double *out)
{
    __shared__ double red[BS / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = red[0];
#pragma unroll
        for (int k = 1; k < BS / 64; k++) s += red[k];
        *out = s;
    }
}

// -------------------------------------------------------------------------
// The 9 FD columns of [A | B] for fix_calibration (NA = 6), shared by the two
// lanes of an observation with one instruction stream and the work each
// column really needs (mex_bundle_1_XABeUVWeAeB.c:14-70, the same
// expressions as project_col):
//   3 "full" rounds   lane 0: rotation column t  -- R(w + h e_t), t + 0, b
//                     lane 1: point column t     -- R(w), t, b + h e_t
//   2 "shift" rounds  translation columns 3, 4 | 5, -: R(w + 0) b is shared
//                     (vlg_rot_b), only S + (t + h e_k) is formed per column
// Every operand is formed exactly as the reference forms it (a0 + h * 0.0 for
// the unperturbed camera components of a camera column, a0 itself for a
// point column), so the columns are bit-identical to project_col's.
// -------------------------------------------------------------------------
__device__ __forceinline__ void fd_columns_6(const cam_view<6> &cv, const double b[3],
                                             const double xh[2], int half, double *row)
{
    const double *t0 = cv.a0 + 3;
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const double *Rs = cv.R + 9 * (half ? 0 : 1 + t);
        double Rk[9], tt[3], bb[3], x1[2], S[3];
#pragma unroll
        for (int q = 0; q < 9; q++) Rk[q] = Rs[q];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            tt[c] = half ? t0[c] : t0[c] + H_FD * 0.0;
            bb[c] = half ? b[c] + H_FD * ((c == t) ? 1.0 : 0.0) : b[c];
        }
        vlg_rot_b(Rk, bb, S);
        vlg_project_s(cv.Kc, S, tt, x1);
        const int col = half ? 6 + t : t;
        row[2 * col] = vlg_fd_quot(x1[0] - xh[0]);
        row[2 * col + 1] = vlg_fd_quot(x1[1] - xh[1]);
    }
    double S[3], R4[9];
    const double *Rs4 = cv.R + 36;
#pragma unroll
    for (int q = 0; q < 9; q++) R4[q] = Rs4[q];
    vlg_rot_b(R4, b, S);
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int k = 3 + 2 * u + half;      // 3, 4 | 5, (6: idle)
        if (k < 6) {
            double tt[3], x1[2];
#pragma unroll
            for (int c = 0; c < 3; c++) tt[c] = t0[c] + H_FD * ((3 + c == k) ? 1.0 : 0.0);
            vlg_project_s(cv.Kc, S, tt, x1);
            row[2 * k] = vlg_fd_quot(x1[0] - xh[0]);
            row[2 * k + 1] = vlg_fd_quot(x1[1] - xh[1]);
        }
    }
}

template <int NA>
__global__ void k_rotations(const double *__restrict__ a, double *__restrict__ rot, int m)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const double *aj = a + (size_t)NA * j;
    const double w[3] = {aj[0], aj[1], aj[2]};
    rotations5(w, rot + 45 * (size_t)j);
}

// device sin / cos of the rotations (vlg_libm.h), exported for the parity
// test that compares them with the host libm (vlgba_debug_sincos)
__global__ void k_sincos(const double *__restrict__ x, double *__restrict__ s,
                         double *__restrict__ c, long long n)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    s[i] = vlg_lm_sin(v);
    c[i] = vlg_lm_cos(v);
}

extern "C" int vlgba_debug_sincos(const double *x, double *s, double *c, long long n)
{
    if (n < 0 || (n > 0 && (!x || !s || !c))) return VLGBA_E_ARG;
    if (n == 0) return 0;
    double *d = nullptr;
    VLGBA_CHECK(hipMalloc(&d, sizeof(double) * 3 * (size_t)n));
    int rc = 0;
    do {
        if (hipMemcpy(d, x, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) { rc = -1; break; }
        const long long nb = (n + 255) / 256;
        hipLaunchKernelGGL(k_sincos, dim3((unsigned)nb), dim3(256), 0, 0, d, d + n, d + 2 * n, n);
        if (hipGetLastError() != hipSuccess) { rc = -1; break; }
        if (hipMemcpy(s, d + n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(c, d + 2 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess)
            rc = -1;
    } while (0);
    (void)hipFree(d);
    return rc;
}

// -------------------------------------------------------------------------
// linearisation, one thread per point (observations in ascending camera order)
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(256) void k_linearize(
    const int *__restrict__ pt_ptr, const int *__restrict__ obs_cam,
    const double *__restrict__ obs_x, const double *__restrict__ K4,
    const double *__restrict__ a, const double *__restrict__ rot,
    const double *__restrict__ b, int n, ba_flags f, const unsigned char *__restrict__ pivot,
    double *__restrict__ jrec, double *__restrict__ W, double *__restrict__ V,
    double *__restrict__ eB, double *__restrict__ part_sse, double *__restrict__ xh_out,
    double *__restrict__ B_out)
{
    constexpr int JS = 2 * NA + 2;
    double sse = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double bi[3] = {b[3 * (size_t)i], b[3 * (size_t)i + 1], b[3 * (size_t)i + 2]};
        double v[9], eb[3];
#pragma unroll
        for (int q = 0; q < 9; q++) v[q] = 0.0;
        eb[0] = eb[1] = eb[2] = 0.0;
        const int o_end = pt_ptr[i + 1];
        for (int o = pt_ptr[i]; o < o_end; o++) {
            const int j = obs_cam[o];
            cam_view<NA> cv(a, K4, rot, j);
            double xh[2];
            cv.project(bi, xh);
            double A[2 * NA], B[6];
            // camera derivatives, mex_bundle_1_XABeUVWeAeB.c:201-209, 14-41
            // (mex_bundle_proj_1_XABeUVWeAeB.c:204-211, 34-59)
#pragma unroll
            for (int k = 0; k < NA; k++) {
                double x1[2];
                cv.project_dcam(k, bi, x1);
                A[2 * k] = vlg_fd_quot(x1[0] - xh[0]);
                A[2 * k + 1] = vlg_fd_quot(x1[1] - xh[1]);
            }
            // point derivatives, :211-219, 43-70 (proj :214-221, 61-86)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                double b1[3], x1[2];
#pragma unroll
                for (int c = 0; c < 3; c++) b1[c] = bi[c] + H_FD * ((c == k) ? 1.0 : 0.0);
                cv.project(b1, x1);
                B[2 * k] = vlg_fd_quot(x1[0] - xh[0]);
                B[2 * k + 1] = vlg_fd_quot(x1[1] - xh[1]);
            }
            const double e0 = obs_x[2 * (size_t)o] - xh[0];
            const double e1 = obs_x[2 * (size_t)o + 1] - xh[1];
            double *rec = jrec + (size_t)JS * o;
#pragma unroll
            for (int q = 0; q < 2 * NA; q += 2) {
                double2 p = {A[q], A[q + 1]};
                *reinterpret_cast<double2 *>(rec + q) = p;
            }
            *reinterpret_cast<double2 *>(rec + 2 * NA) = double2{e0, e1};
            if (xh_out) {
                xh_out[2 * (size_t)o] = xh[0];
                xh_out[2 * (size_t)o + 1] = xh[1];
            }
            if (B_out) {
#pragma unroll
                for (int q = 0; q < 6; q++) B_out[6 * (size_t)o + q] = B[q];
            }
            // W_ij = A^T B onto a zeroed output (:305-314)
            const bool wzero = f.fix_structure || f.fix_motion || (f.has_pivot && pivot[j]);
            double *wo = W + (size_t)3 * NA * o;
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int r = 0; r < NA; r++)
                    wo[r + NA * c] =
                        wzero ? 0.0 : 0.0 + (A[2 * r] * B[2 * c] + A[2 * r + 1] * B[2 * c + 1]);
            // V_i += B^T B, eB_i += B^T e (:293-302, :326-332)
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int r = 0; r < 3; r++)
                    v[r + 3 * c] += B[2 * r] * B[2 * c] + B[2 * r + 1] * B[2 * c + 1];
#pragma unroll
            for (int r = 0; r < 3; r++) eb[r] += B[2 * r] * e0 + B[2 * r + 1] * e1;
            sse += e0 * e0 + e1 * e1;
        }
        if (f.fix_structure) {
#pragma unroll
            for (int q = 0; q < 9; q++) v[q] = 0.0;
            eb[0] = eb[1] = eb[2] = 0.0;
        }
#pragma unroll
        for (int q = 0; q < 9; q++) V[9 * (size_t)i + q] = v[q];
#pragma unroll
        for (int q = 0; q < 3; q++) eB[3 * (size_t)i + q] = eb[q];
    }
    block_sum_to<256>(sse, part_sse + blockIdx.x);
}

// -------------------------------------------------------------------------
// Fast-path linearisation, one workgroup per Schur chunk (<= 128 observations
// of consecutive points), two lanes per observation: both project the base
// point, then lane 0 the first NC0 of the NA + 3 FD columns of [A | B] and
// lane 1 the rest, through one branch-free column routine (same expressions
// as k_linearize), so the wave runs 1 + NC0 projections, not 1 + NA + 3.
// A, B, e go to LDS; then per observation W_ij (one contiguous,
// coalesced HBM range per chunk), per point V_i / eB_i (sequential over the
// point's cameras, as k_linearize), per camera of the chunk one partial of
// U_j / eA_j (sequential over the chunk's points), reduced per camera in chunk
// order by k_camera_reduce_chunks.  jrec is never written.
// -------------------------------------------------------------------------
// 7 waves per SIMD for NA = 6: the LDS rows (21.7 KB) allow 7 workgroups per
// CU; the bound keeps the register allocation from costing one of them
#ifndef BA_LIN_W2_ON
#define BA_LIN_W2_ON 1
#endif

// UPD = true (k_update_linearize): the point update of the pass that just
// solved (mex_bundle_3_db_new.c:99-146: db_i, b_new, the point part of
// dp'(lambda dp + g)) runs first in the same workgroup, from the pass's W / eB
// / V*^-1 (double-buffered: they stay valid for a rejected step), and the
// chunk is then linearised at (a_new, b_new) into the other buffers -- whose
// base projection IS the update's new projection (:149-166), so its SSE is
// the pass's new SSE and, if the step is accepted, the next pass's old SSE
// (bundle_euclid.m:139 of the next iteration recomputes exactly that, App. A
// Q12).  One pass over the observations instead of two.
// BA_LIN_CAMS (NA = 6): the rotation-table rows (45 doubles) of the chunk's
// cameras -- a chunk of consecutive points sees a narrow camera range, ~7
// cameras at config 3 -- staged in LDS by LDS-DMA with the chunk's other
// operands, so the projections read R(w), R(w + h e_k), R(w + 0) from LDS
// instead of every lane fetching its camera's 360 bytes of them through the
// vector-memory path (the kernel's busiest unit: TD 90 %, TA 80 % busy,
// profiles/r06/pmc_cfg3_summary.csv): 298 -> 277-279 us at config 3
// (profiles/r06/ab_lin_cams.txt).  Chunks whose cameras span more than
// BA_LIN_CAMS read the table from memory as before.  The same values: bit for
// bit the same columns.  (Staging a and K4 as well measured 326-328 us.)  0: off.
#ifndef BA_LIN_CAMS
#define BA_LIN_CAMS 10
#endif
// waves per SIMD the NA = 6 linearisation kernels are compiled for: 6 with the
// staged cameras (80 VGPRs; their LDS allows 6 workgroups per CU), else 7 (72
// VGPRs, 7 workgroups per CU)
#ifndef BA_LIN_WAVES
#define BA_LIN_WAVES (BA_LIN_CAMS > 0 ? 6 : 7)
#endif

struct ba_upd {
    const double *W_old, *da, *eB_old, *Vinv, *b_old;
    int ndb;
    double lambda;
    double *db, *b_new, *part_dpg;
    const int *seg_long, *long_o0;
    const double *dpg_long;
};

template <int NA, bool UPD>
__device__ __forceinline__ void linearize_chunk_body(
    const int *__restrict__ ch_pt, const int *__restrict__ ch_obase,
    const int *__restrict__ ch_eslot, const int *__restrict__ eslot_optr,
    const unsigned short *__restrict__ eslot_obs, const int *__restrict__ pt_ptr,
    const int *__restrict__ obs_cam, const unsigned char *__restrict__ obs_lpt,
    const double *__restrict__ obs_x, const double *__restrict__ K4,
    const double *__restrict__ a, const double *__restrict__ rot,
    const double *__restrict__ b, ba_flags f, const unsigned char *__restrict__ pivot,
    double *__restrict__ W, double *__restrict__ V, double *__restrict__ eB,
    double *__restrict__ upart, double *__restrict__ part_sse, int nch_reg,
    const int *__restrict__ seg_pt, double *__restrict__ vseg, const int *__restrict__ ch_cam,
    ba_upd u, int ch)
{
    constexpr int NC0 = (NA + 4) / 2;       // lane 0: base + FD columns [0, NC0)
    constexpr int RS = 2 * NA + 8;          // LDS row: A (2 NA), B (6), e (2)
    constexpr int NU = NA * (NA + 1) / 2;
    static_assert(BA_CH_OBS + 1 <= 256 && BA_CH_PTS + 1 <= 256, "one metadata word per lane");
    // UPD: the rows hold the chunk's old W rows, then t_o, with the new points
    // b_new after them (LW), before they take A, B, e (NA = 6: the same 20 KB,
    // so 7 workgroups per CU still fit)
    constexpr int LW = BA_CH_OBS * 3 * NA;
    constexpr int NROWS = (UPD && LW + 3 * BA_CH_PTS > BA_CH_OBS * RS) ? LW + 3 * BA_CH_PTS
                                                                        : BA_CH_OBS * RS;
    static_assert(NA != 6 || NROWS == BA_CH_OBS * RS, "fused update must not grow NA = 6 LDS");
    __shared__ __attribute__((aligned(16))) double rows[NROWS];
    // pt_ptr[p0 + t] (t <= np) and eslot_optr[e0 + t] (t <= nes) as they are
    // in memory, written by LDS-DMA (no registers, no wait until the barrier)
    // from the waves whose lanes cover them
    __shared__ int lptr_raw[64 * (BA_CH_PTS / 64 + 1)];
    __shared__ int eoff_raw[64 * (BA_CH_OBS / 64 + 1)];
    __shared__ unsigned short eobl[BA_CH_OBS];
    __shared__ unsigned char wz[BA_CH_OBS]; // W_ij forced to zero (fix masks, :140-154)
    // UPD: the point lanes' dp'(lambda dp + g) terms (wave 0), summed by
    // thread 0 after the projections (a shuffle reduction here would keep its
    // lane addresses live through the projections: spills)
    __shared__ double dpl[UPD ? BA_CH_PTS : 1];
    static_assert(BA_CH_PTS <= 64, "the point lanes are wave 0");
    // the chunk's rotation-table rows (BA_LIN_CAMS cameras)
    constexpr int NCAMS = (NA == 6 && BA_LIN_CAMS > 0) ? BA_LIN_CAMS : 0;
    __shared__ __attribute__((aligned(16))) double camr[NCAMS > 0 ? 45 * NCAMS : 1];
    const int tid = threadIdx.x;
    // a segment chunk (ch >= nch_reg) holds part of one long track: its V / eB
    // sums are partials (vseg), added up per track by k_long_vsum
    const bool seg = ch >= nch_reg;
    const int p0 = seg ? seg_pt[ch - nch_reg] : ch_pt[ch];
    const int np = seg ? 1 : ch_pt[ch + 1] - p0;
    const int obase = ch_obase[ch], nobs = ch_obase[ch + 1] - obase;
    const int e0 = ch_eslot[ch], nes = ch_eslot[ch + 1] - e0;
    STAMP_DECL;
    // Metadata of the reduction phases: loaded now, stored to LDS after the
    // projections, so its dependent loads ride along with the observation and
    // camera loads instead of adding round trips (and a barrier) up front.
    // Every load of this prologue and of the projections' operands is
    // issued by every lane at a clamped, valid index (no divergent branch
    // around a load: the compiler then waits on each one before the next
    // block), so the dependent chains overlap.
    const int u0 = eslot_optr[e0], nu = eslot_optr[e0 + nes] - u0;
    {
        const int wv = tid >> 6;   // uniform per wave
        if (wv <= (nes >> 6))
            __builtin_amdgcn_global_load_lds(eslot_optr + e0 + min(tid, nes), eoff_raw + 64 * wv,
                                             4, 0, 0);
        if (!seg && wv <= (np >> 6))
            __builtin_amdgcn_global_load_lds(pt_ptr + p0 + min(tid, np), lptr_raw + 64 * wv, 4, 0,
                                             0);
    }
    // the chunk's camera range (ch_cam: lowest / highest camera of the chunk)
    const int cam_lo = ch_cam[2 * ch], cam_n = ch_cam[2 * ch + 1] - cam_lo + 1;
    const bool camst = NCAMS > 0 && nobs > 0 && cam_n <= NCAMS;   // (uniform)
    if (NCAMS > 0 && camst) {
#if defined(__HIP_DEVICE_COMPILE__)
        // one contiguous range, one dword per lane (exec-masked past its end)
        const int lane = tid & 63;
        auto stage = [&](const double *src, int ndw, double *dst) {
            const char *s8 = reinterpret_cast<const char *>(src);
            for (int q = tid >> 6; 64 * q < ndw; q += 4)   // (wave-uniform)
                if (64 * q + lane < ndw)
                    __builtin_amdgcn_global_load_lds(s8 + 4 * (64 * q + lane),
                                                     reinterpret_cast<int *>(dst) + 64 * q, 4, 0,
                                                     0);
        };
        stage(rot + 45 * (size_t)cam_lo, 90 * cam_n, &camr[0]);
#endif
        if constexpr (!UPD) __syncthreads();   // (UPD: the update's barriers)
    }
    int m_eobl = 0;
    STAMP(16);
    double bu[3] = {0.0, 0.0, 0.0};   // UPD: this lane's point at b_new
    if constexpr (UPD) {
        // ---- the update (k_point_update_chunk's arithmetic, same order) ----
        if (seg) {   // a long track's segment: db / b_new / dp'g by k_long_db
            if (tid == 0)
                dpl[0] = obase == u.long_o0[u.seg_long[ch - nch_reg]]
                             ? __hip_atomic_load(u.dpg_long + u.seg_long[ch - nch_reg],
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0.0;
        } else {
            const int ne = nobs * 3 * NA;
            const double *wsrc = u.W_old + (size_t)3 * NA * obase;
            double dl[NA];
            const int ocam = nobs > 0 ? obs_cam[obase + min(tid, nobs - 1)] : 0;
            // the da rows of the chunk's cameras (a narrow range: consecutive
            // points see neighbouring cameras) by LDS-DMA into the row area's
            // tail, beside the W rows: the lanes index them with their camera
            // after the barrier, so no load waits on another.  A wider range
            // loads each lane's da row from its camera index (dependent).
            const int clo = cam_lo, span = cam_n;
            const bool dstage = NA == 6 && span * NA <= NROWS - LW;
            if (dstage && nobs > 0) {
#if defined(__HIP_DEVICE_COMPILE__)
                const int nb = 8 * NA * span;
                if ((tid >> 6) < ((nb + 1023) >> 10))
                    __builtin_amdgcn_global_load_lds(
                        reinterpret_cast<const char *>(u.da + (size_t)NA * clo) +
                            min((tid >> 6) * 1024 + 16 * (tid & 63), nb - 16),
                        &rows[LW + 128 * (tid >> 6)], 16, 0, 0);
#endif
            }
            if (nobs > 0) {
                if constexpr (NA == 6) {
                    // the chunk's old W rows (one contiguous range, 144 B per
                    // observation: 16-byte aligned) straight into LDS by LDS-DMA,
                    // 1 KiB per wave-instruction, non-temporal (W's last reader):
                    // no registers, in flight until the barrier below
                    // (the 16-byte form exists for gfx950 only: the host pass of
                    // the compiler would drop the kernel's launch stub over it)
#if defined(__HIP_DEVICE_COMPILE__)
                    const int nbytes = 8 * ne, ninst = (nbytes + 1023) >> 10;
                    const char *src = reinterpret_cast<const char *>(wsrc);
                    for (int q = tid >> 6; q < ninst; q += 4)
                        __builtin_amdgcn_global_load_lds(
                            src + min(q * 1024 + 16 * (tid & 63), nbytes - 16), &rows[128 * q],
                            16, 0, 2);
#endif
                } else {
                    constexpr int MAXE = (LW + 255) / 256;
#pragma unroll
                    for (int q = 0; q < MAXE; q++) {
                        const int e = tid + 256 * q;
                        if (e < ne) rows[e] = __builtin_nontemporal_load(wsrc + e);
                    }
                }
                if (!dstage) {
                    const double *dd = u.da + (size_t)NA * ocam;
#pragma unroll
                    for (int k = 0; k < NA; k++) dl[k] = dd[k];
                }
            }
            // the point lanes' operands (eB, V*^-1, b): in flight through t_o;
            // wave 0 only (the point lanes, np <= 64; wave-uniform): the
            // other waves' clamped copies were TD-path traffic for nothing
            // (the kernel's vector-memory data path is its busiest unit, TD
            // busy 90 %: 316 -> 298-301 us, profiles/r06/ab_lin.txt)
            const int ip = np > 0 ? p0 + min(tid, np - 1) : 0;
            double pe[3] = {0.0, 0.0, 0.0}, pv[9] = {}, pb[3] = {0.0, 0.0, 0.0};
            if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
#pragma unroll
                for (int r = 0; r < 3; r++) pe[r] = u.eB_old[3 * (size_t)ip + r];
#pragma unroll
                for (int r = 0; r < 9; r++) pv[r] = u.Vinv[9 * (size_t)ip + r];
#pragma unroll
                for (int r = 0; r < 3; r++) pb[r] = u.b_old[3 * (size_t)ip + r];
            }
            __syncthreads();
            // t_o[r] = W_o(:, r)' da_j (mex_bundle_3_db_new.c:113-120), into the
            // row's first slot (only this lane reads the row)
            if (tid < nobs) {
                double *wo = rows + 3 * NA * tid;
                if (dstage) {
#pragma unroll
                    for (int k = 0; k < NA; k++) dl[k] = rows[LW + NA * (ocam - clo) + k];
                }
#pragma unroll
                for (int k = 0; k < NA; k++)   // da(1:ndb) only (mex_bundle_3 :113-120)
                    if (k >= u.ndb) dl[k] = 0.0;
#pragma unroll
                for (int r = 0; r < 3; r++) {
                    double *w = wo + NA * r;
                    double t = w[0] * dl[0] + w[1] * dl[1] + w[2] * dl[2] + w[3] * dl[3] +
                               w[4] * dl[4] + w[5] * dl[5];
#pragma unroll
                    for (int k = 6; k < NA; k++)   // nomex semantics only (ndb = NA)
                        if (k < u.ndb) t = t + w[k] * dl[k];
                    w[0] = t;
                }
            }
            __syncthreads();
            // rhs = eB_i - t_o1 - t_o2 - ... (cameras ascending), db_i = V*_i^-1 rhs,
            // b_new, dp'(lambda dp + g) (:99-146, bundle_euclid.m:213-217); a
            // point without observations gets db = V*^-1 eB (= 0) all the same
            if (tid < np) {
                const int i = p0 + tid;
                double rhs[3] = {pe[0], pe[1], pe[2]};
                const int lo1 = lptr_raw[tid + 1] - obase;
                for (int lo = lptr_raw[tid] - obase; lo < lo1; lo++) {
#pragma unroll
                    for (int r = 0; r < 3; r++) rhs[r] -= rows[3 * NA * lo + NA * r];
                }
                double dpg = 0.0;
#pragma unroll
                for (int r = 0; r < 3; r++) {
                    const double dbr = pv[r] * rhs[0] + pv[r + 3] * rhs[1] + pv[r + 6] * rhs[2];
                    const double bnr = pb[r] + dbr;
                    u.db[3 * (size_t)i + r] = dbr;
                    u.b_new[3 * (size_t)i + r] = bnr;
                    rows[LW + 3 * tid + r] = bnr;   // (after every t_o read: barrier B)
                    dpg += dbr * (u.lambda * dbr + pe[r]);
                }
                dpl[tid] = dpg;
            }
        }
        __syncthreads();
        // every lane takes its observation's b_new from LDS (a long track's
        // segment: from k_long_db's b_new) before the projections overwrite the
        // rows
        if (!seg && nobs > 0) {
            const int lp = obs_lpt[obase + min(min(tid >> 1, BA_CH_OBS - 1), nobs - 1)];
#pragma unroll
            for (int c = 0; c < 3; c++) bu[c] = rows[LW + 3 * lp + c];
        } else if (nobs > 0) {
#pragma unroll
            for (int c = 0; c < 3; c++) bu[c] = b[3 * (size_t)p0 + c];
        }
        __syncthreads();
        STAMP(23);
    }
    double sse = 0.0;
    if (nobs > 0) {   // (nu > 0 too)
        m_eobl = __hip_atomic_load(eslot_obs + u0 + min(tid, nu - 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        // lanes past the chunk's observations project its last one again
        // into rows nobs .. BA_CH_OBS - 1, which nothing reads (lanes past
        // BA_CH_OBS rows, when it is < 128, into the last row: the same
        // values as any lane that writes it)
        const int lo = min(tid >> 1, BA_CH_OBS - 1), half = tid & 1;
        const bool live = (tid >> 1) < nobs;
        {
            const int o = obase + min(lo, nobs - 1);
            const int j = obs_cam[o], i = p0 + obs_lpt[o];
            double bi[3];
#pragma unroll
            for (int c = 0; c < 3; c++) bi[c] = UPD ? bu[c] : b[3 * (size_t)i + c];
            double xh[2];
            double *row = rows + RS * lo;
            if constexpr (NA == 6) {
                // the rotations from LDS (staged) or the table: one code path
                // each, so every load has its address space at compile time
                auto proj6 = [&](const double *rt, int jr) {
                    cam_view<NA> cv6(a, K4, rt, jr, j);
                    cv6.project(bi, xh);
                    fd_columns_6(cv6, bi, xh, half, row);
                };
                if (NCAMS > 0 && camst)
                    proj6(&camr[0], j - cam_lo);
                else
                    proj6(rot, j);
            } else {
                cam_view<NA> cv(a, K4, rot, j);
                cv.project(bi, xh);
                // the NA + 3 FD columns of [A | B] (mex_bundle_1 :201-219) split
                // evenly: lane 0 columns [0, NC0), lane 1 [NC0, NA + 3), one
                // instruction stream for both (project_col has no branch)
#pragma unroll 1
                for (int t = 0; t < NC0; t++) {
                    const int col = half ? NC0 + t : t;
                    if (col < NA + 3) {
                        double x1[2];
                        cv.project_col(col, bi, x1);
                        row[2 * col] = vlg_fd_quot(x1[0] - xh[0]);
                        row[2 * col + 1] = vlg_fd_quot(x1[1] - xh[1]);
                    }
                }
            }
            if (!half) {
                const double e0 = obs_x[2 * (size_t)o] - xh[0];
                const double e1 = obs_x[2 * (size_t)o + 1] - xh[1];
                row[2 * NA + 6] = e0;
                row[2 * NA + 7] = e1;
                if (live) sse = e0 * e0 + e1 * e1;
                wz[lo] = f.fix_structure || f.fix_motion || (f.has_pivot && pivot[j]);
            }
        }
    }
    if (tid < nu) eobl[tid] = (unsigned short)m_eobl;
    __syncthreads();
    STAMP(17);
    if constexpr (UPD) {   // the chunk's point part of dp'(lambda dp + g), points in order
        if (tid == 0) {
            double acc = 0.0;
            const int k1 = seg ? 1 : np;
            for (int k = 0; k < k1; k++) acc += dpl[k];
            u.part_dpg[ch] = acc;
        }
    }
    // W_ij = A^T B onto a zeroed output (:305-314): the chunk's W rows are one
    // contiguous HBM range, written lane by lane (coalesced), two entries
    // (rows r, r + 1 of one column) per lane
    if constexpr (BA_LIN_W2_ON && NA % 2 == 0) {
        double2 *wdst = reinterpret_cast<double2 *>(W + (size_t)3 * NA * obase);
        constexpr int NP = 3 * NA / 2;         // entry pairs per observation
        for (int q = tid; q < nobs * NP; q += 256) {
            const int lo = q / NP, e = q - NP * lo, c = e / (NA / 2), r = 2 * (e - (NA / 2) * c);
            const double *row = rows + RS * lo;
            const double2 a0 = *reinterpret_cast<const double2 *>(row + 2 * r);
            const double2 a1 = *reinterpret_cast<const double2 *>(row + 2 * r + 2);
            const double2 bc = *reinterpret_cast<const double2 *>(row + 2 * NA + 2 * c);
            const long long keep = wz[lo] ? 0 : -1;   // forced zeros by a mask, no branch
            const double v0 = 0.0 + (a0.x * bc.x + a0.y * bc.y);
            const double v1 = 0.0 + (a1.x * bc.x + a1.y * bc.y);
            // streamed (non-temporal): W is re-read only after the whole 432 MB
            // (config 3) has been written, so caching it only evicts the
            // observation / camera / point data of the next workgroups
            const v2d w2 = {__builtin_bit_cast(double, __builtin_bit_cast(long long, v0) & keep),
                            __builtin_bit_cast(double, __builtin_bit_cast(long long, v1) & keep)};
            __builtin_nontemporal_store(w2, reinterpret_cast<v2d *>(wdst) + q);
        }
    } else {
        double *wdst = W + (size_t)3 * NA * obase;
        for (int q = tid; q < nobs * 3 * NA; q += 256) {
            const int lo = q / (3 * NA), e = q - 3 * NA * lo, c = e / NA, r = e - NA * c;
            const double *row = rows + RS * lo;
            const double2 ar = *reinterpret_cast<const double2 *>(row + 2 * r);
            const double2 bc = *reinterpret_cast<const double2 *>(row + 2 * NA + 2 * c);
            wdst[q] = wz[lo] ? 0.0 : 0.0 + (ar.x * bc.x + ar.y * bc.y);
        }
    }
    STAMP(18);
    // V_i += B^T B, eB_i += B^T e over the point's cameras (:293-302, :326-332)
    for (int q = tid; q < np * 12; q += 256) {
        const int pl = q / 12, e = q % 12, i = p0 + pl;
        const int lo0 = seg ? 0 : lptr_raw[pl] - obase;
        const int lo1 = seg ? nobs : lptr_raw[pl + 1] - obase;
        // one loop for both kinds (no divergent pair of loops in a wave): e
        // is the column after B's three, B[6], B[7]
        const int r = (e < 9) ? e % 3 : e - 9, c = (e < 9) ? e / 3 : 3;
        double acc = 0.0;
        for (int lo = lo0; lo < lo1; lo++) {
            const double *B = rows + RS * lo + 2 * NA;
            acc += B[2 * r] * B[2 * c] + B[2 * r + 1] * B[2 * c + 1];
        }
        if (f.fix_structure) acc = 0.0;
        if (seg) vseg[12 * (size_t)(ch - nch_reg) + e] = acc;
        else if (e < 9) V[9 * (size_t)i + e] = acc;
        else eB[3 * (size_t)i + e - 9] = acc;
    }
    STAMP(19);
    // U_j (lower triangle) / eA_j partials per camera of the chunk
    for (int q = tid; q < nes * (NU + NA); q += 256) {
        const int s = q / (NU + NA), l = q % (NU + NA);
        int r, c;
        if (l < NU) {
            int t = l;
            c = 0;
            while (t >= NA - c) { t -= NA - c; c++; }
            r = c + t;
        } else {
            r = l - NU;
            c = NA;   // e occupies the column after B: row[2 NA + 6]
        }
        const int cc = (c < NA) ? 2 * c : 2 * NA + 6;
        // four observations a step: their index and data reads in flight
        // together, the sum still taken one observation at a time in order
        double acc = 0.0;
        int u = eoff_raw[s] - u0;
        const int u1 = eoff_raw[s + 1] - u0;
        for (; u + 3 < u1; u += 4) {
            double p[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const double *rw = rows + RS * eobl[u + k];
                p[k] = rw[2 * r] * rw[cc] + rw[2 * r + 1] * rw[cc + 1];
            }
#pragma unroll
            for (int k = 0; k < 4; k++) acc += p[k];
        }
        for (; u < u1; u++) {
            const double *row = rows + RS * eobl[u];
            acc += row[2 * r] * row[cc] + row[2 * r + 1] * row[cc + 1];
        }
        upart[(size_t)(NU + NA) * (e0 + s) + l] = acc;
    }
    STAMP(20);
    block_sum_to<256>(sse, part_sse + ch);
    STAMP(21);
#ifdef BA_STAMPS
    if (tid == 0) atomicAdd(&g_stamp[22], 1ull);
#endif
}

#define BA_LIN_ARGS                                                                        \
    const int *__restrict__ ch_pt, const int *__restrict__ ch_obase,                       \
        const int *__restrict__ ch_eslot, const int *__restrict__ eslot_optr,              \
        const unsigned short *__restrict__ eslot_obs, const int *__restrict__ pt_ptr,      \
        const int *__restrict__ obs_cam, const unsigned char *__restrict__ obs_lpt,        \
        const double *__restrict__ obs_x, const double *__restrict__ K4,                   \
        const double *__restrict__ a, const double *__restrict__ rot,                      \
        const double *__restrict__ b, ba_flags f, const unsigned char *__restrict__ pivot, \
        double *__restrict__ W, double *__restrict__ V, double *__restrict__ eB,           \
        double *__restrict__ upart, double *__restrict__ part_sse, int nch_reg,            \
        const int *__restrict__ seg_pt, double *__restrict__ vseg,                         \
        const int *__restrict__ ch_cam
#define BA_LIN_PASS                                                                        \
    ch_pt, ch_obase, ch_eslot, eslot_optr, eslot_obs, pt_ptr, obs_cam, obs_lpt, obs_x, K4, a, \
        rot, b, f, pivot, W, V, eB, upart, part_sse, nch_reg, seg_pt, vseg, ch_cam

// the linearisation at the current parameters (after set_params, the ordered
// and stage paths' fast twin)
template <int NA>
__global__ __launch_bounds__(256, (NA == 6) ? BA_LIN_WAVES : 1) void k_linearize_chunk(BA_LIN_ARGS)
{
    linearize_chunk_body<NA, false>(BA_LIN_PASS, ba_upd{}, blockIdx.x);
}

// the fused update: the point update of the pass, then the linearisation at
// (a_new, b_new) (a, rot, b = a_new, rot_new, b_new; W .. part_sse = the
// second buffers)
template <int NA>
__global__ __launch_bounds__(256, (NA == 6) ? BA_LIN_WAVES : 1) void k_update_linearize(BA_LIN_ARGS,
                                                                             ba_upd u)
{
    linearize_chunk_body<NA, true>(BA_LIN_PASS, u, blockIdx.x);
}

// U_j, eA_j from the per-chunk partials (fast path).  One 256-lane workgroup
// per camera: lane (entry l, stream p) sums the camera's partials p, p + P,
// p + 2P, ... (P = 256 / (NU + NA) streams, so ~P loads are in flight per
// entry instead of one dependent chain); the streams are then added in
// stream order.  Fixed order -> deterministic run to run.
// workgroup j of the camera reduction (j == m: the SSE)
template <int NA>
__device__ __forceinline__ void camera_reduce_wg(int j, const ba_camred &a)
{
    const int *__restrict__ cam_eptr = a.cam_eptr;
    const int *__restrict__ cam_eslots = a.cam_eslots;
    const double *__restrict__ upart = a.upart;
    const int m = a.m, nch = a.nch;
    const ba_flags f = a.f;
    const unsigned char *__restrict__ pivot = a.pivot;
    double *__restrict__ U = a.U;
    double *__restrict__ eA = a.eA;
    const double *__restrict__ chsse = a.chsse;
    double *__restrict__ sse_out = a.sse_out;
    double *__restrict__ sse_out2 = a.sse_out2;
    constexpr int NU = NA * (NA + 1) / 2;
    constexpr int NT = NU + NA;
    constexpr int P = 256 / NT;
    __shared__ double part[P][NT];
    const int tid = threadIdx.x;
    if (j == m) {   // extra workgroup: the linearisation SSE (old_error), fixed order
        double v[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        int q = tid;
        for (; q + 7 * 256 < nch; q += 8 * 256) {
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] += chsse[q + 256 * u];
        }
        for (; q < nch; q += 256) v[0] += chsse[q];
        block_sum_to<256>(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])),
                          sse_out);
        if (tid == 0) sse_out2[0] = sse_out[0];
        return;
    }
    const int l = tid % NT, p = tid / NT;
    if (p < P) {
        const int q0 = cam_eptr[j], q1 = cam_eptr[j + 1];
        // four partials of the stream a step: their index and value loads in
        // flight together (a dependent pair of L2 round trips per partial
        // otherwise), added in stream order
        double acc = 0.0;
        int q = q0 + p;
        for (; q + 3 * P < q1; q += 4 * P) {
            int ix[4];
            double v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) ix[k] = cam_eslots[q + k * P];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = upart[(size_t)NT * ix[k] + l];
#pragma unroll
            for (int k = 0; k < 4; k++) acc += v[k];
        }
        for (; q < q1; q += P) acc += upart[(size_t)NT * cam_eslots[q] + l];
        part[p][l] = acc;
    }
    __syncthreads();
    if (tid >= NT) return;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < P; k++) acc += part[k][tid];
    if (f.fix_motion || (f.has_pivot && pivot[j])) acc = 0.0;
    if (tid < NU) {
        int t = tid, c = 0;
        while (t >= NA - c) { t -= NA - c; c++; }
        const int r = c + t;
        U[(size_t)NA * NA * j + r + NA * c] = acc;
        U[(size_t)NA * NA * j + c + NA * r] = acc;
    } else {
        eA[(size_t)NA * j + tid - NU] = acc;
    }
}

template <int NA>
__global__ __launch_bounds__(256) void k_camera_reduce_chunks(ba_camred a)
{
    camera_reduce_wg<NA>(blockIdx.x, a);
}

// -------------------------------------------------------------------------
// U_j, eA_j: one workgroup per camera, each output owned by one lane and
// summed sequentially over the camera's observations in ascending point order
// (= mex_bundle_1_XABeUVWeAeB.c:266-323 with the exact zeros skipped).
// -------------------------------------------------------------------------
template <int NA>
__global__ void k_camera_reduce(const int *__restrict__ cam_ptr, const int *__restrict__ cam_obs,
                                const double *__restrict__ jrec, int m, ba_flags f,
                                const unsigned char *__restrict__ pivot, double *__restrict__ U,
                                double *__restrict__ eA)
{
    constexpr int JS = 2 * NA + 2;
    constexpr int NU = NA * (NA + 1) / 2;
    const int j = blockIdx.x;
    const int l = threadIdx.x;
    if (j >= m || l >= NU + NA) return;
    int r, c;
    if (l < NU) {  // lower-triangle entry (r >= c)
        int q = l;
        c = 0;
        while (q >= NA - c) { q -= NA - c; c++; }
        r = c + q;
    } else {       // eA entry: column "c" = the residual slot
        r = l - NU;
        c = NA;
    }
    const int s0 = cam_ptr[j], s1 = cam_ptr[j + 1];
    double acc = 0.0;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
        const double *p0 = jrec + (size_t)JS * cam_obs[s];
        const double *p1 = jrec + (size_t)JS * cam_obs[s + 1];
        const double *p2 = jrec + (size_t)JS * cam_obs[s + 2];
        const double *p3 = jrec + (size_t)JS * cam_obs[s + 3];
        const double x00 = p0[2 * r], x01 = p0[2 * r + 1], y00 = p0[2 * c], y01 = p0[2 * c + 1];
        const double x10 = p1[2 * r], x11 = p1[2 * r + 1], y10 = p1[2 * c], y11 = p1[2 * c + 1];
        const double x20 = p2[2 * r], x21 = p2[2 * r + 1], y20 = p2[2 * c], y21 = p2[2 * c + 1];
        const double x30 = p3[2 * r], x31 = p3[2 * r + 1], y30 = p3[2 * c], y31 = p3[2 * c + 1];
        acc += x00 * y00 + x01 * y01;
        acc += x10 * y10 + x11 * y11;
        acc += x20 * y20 + x21 * y21;
        acc += x30 * y30 + x31 * y31;
    }
    for (; s < s1; s++) {
        const double *p = jrec + (size_t)JS * cam_obs[s];
        acc += p[2 * r] * p[2 * c] + p[2 * r + 1] * p[2 * c + 1];
    }
    if (f.fix_motion || (f.has_pivot && pivot[j])) acc = 0.0;
    if (c < NA) {
        U[(size_t)NA * NA * j + r + NA * c] = acc;
        U[(size_t)NA * NA * j + c + NA * r] = acc;
    } else {
        eA[(size_t)NA * j + r] = acc;
    }
}

// -------------------------------------------------------------------------
// per point, per damping value: V* -> V*^-1, Y_o = W_o V*^-1, t_o = Y_o eB_i
// (bundle_euclid.m:168-184; e_ term of mex_bundle_2_Se_.c:143-147)
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(256) void k_damp_point(
    const int *__restrict__ pt_ptr, const double *__restrict__ V,
    const double *__restrict__ eB, const double *__restrict__ W, int n, double lambda,
    double *__restrict__ Vinv, double *__restrict__ Y, double *__restrict__ t)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        double vs[9], vi[9];
#pragma unroll
        for (int q = 0; q < 9; q++) vs[q] = V[9 * (size_t)i + q];
#pragma unroll
        for (int k = 0; k < 3; k++) vs[4 * k] = (1 + lambda) * vs[4 * k];
        vlg_pinv3(vs, vi);
#pragma unroll
        for (int q = 0; q < 9; q++) Vinv[9 * (size_t)i + q] = vi[q];
        const double eb0 = eB[3 * (size_t)i], eb1 = eB[3 * (size_t)i + 1],
                     eb2 = eB[3 * (size_t)i + 2];
        const int o_end = pt_ptr[i + 1];
        for (int o = pt_ptr[i]; o < o_end; o++) {
            const double *w = W + (size_t)3 * NA * o;
            double *y = Y + (size_t)3 * NA * o;
            double wl[3 * NA], yl[3 * NA];
#pragma unroll
            for (int q = 0; q < 3 * NA; q++) wl[q] = w[q];
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int r = 0; r < NA; r++)
                    yl[r + NA * c] = wl[r] * vi[3 * c] + wl[r + NA] * vi[1 + 3 * c] +
                                     wl[r + 2 * NA] * vi[2 + 3 * c];
#pragma unroll
            for (int q = 0; q < 3 * NA; q++) y[q] = yl[q];
#pragma unroll
            for (int r = 0; r < NA; r++)
                t[(size_t)NA * o + r] = yl[r] * eb0 + yl[r + NA] * eb1 + yl[r + 2 * NA] * eb2;
        }
    }
}

// -------------------------------------------------------------------------
// Schur complement, one workgroup per co-visible block (j >= k):
//   S_jk[r][c] = (j == k ? U*_j[r][c] : 0) - sum_i (Y_ij[r] . W_ik[c])
// each entry summed over the block's points in ascending order
// (mex_bundle_2_Se_.c:80-118).  The diagonal block's workgroup also forms
// e_j = eA_j - sum_i Y_ij eB_i (:132-155).
// -------------------------------------------------------------------------
template <int NA>
__global__ void k_schur(const int *__restrict__ blk_jk, const int *__restrict__ blk_ptr,
                        const int *__restrict__ term, const double *__restrict__ Y,
                        const double *__restrict__ W, const double *__restrict__ t,
                        const double *__restrict__ U, const double *__restrict__ eA, int nb,
                        double lambda, int owner, double *__restrict__ sblk,
                        double *__restrict__ rhs)
{
    const int bk = blockIdx.x;
    const int l = threadIdx.x;
    if (bk >= nb) return;
    const int j = blk_jk[2 * bk], k = blk_jk[2 * bk + 1];
    const int s0 = blk_ptr[bk], s1 = blk_ptr[bk + 1];
    if (l < NA * NA) {
        const int r = l % NA, c = l / NA;
        double acc = 0.0;
        if (j == k && owner) {
            const double u = U[(size_t)NA * NA * j + r + NA * c];
            acc = (r == c) ? (1 + lambda) * u : u;
        }
        int s = s0;
        for (; s + 2 <= s1; s += 2) {
            const double *ya = Y + (size_t)3 * NA * term[2 * s];
            const double *wb = W + (size_t)3 * NA * term[2 * s + 1];
            const double *ya2 = Y + (size_t)3 * NA * term[2 * s + 2];
            const double *wb2 = W + (size_t)3 * NA * term[2 * s + 3];
            const double y0 = ya[r], y1 = ya[r + NA], y2 = ya[r + 2 * NA];
            const double w0 = wb[c], w1 = wb[c + NA], w2 = wb[c + 2 * NA];
            const double z0 = ya2[r], z1 = ya2[r + NA], z2 = ya2[r + 2 * NA];
            const double v0 = wb2[c], v1 = wb2[c + NA], v2 = wb2[c + 2 * NA];
            acc -= y0 * w0 + y1 * w1 + y2 * w2;
            acc -= z0 * v0 + z1 * v1 + z2 * v2;
        }
        for (; s < s1; s++) {
            const double *ya = Y + (size_t)3 * NA * term[2 * s];
            const double *wb = W + (size_t)3 * NA * term[2 * s + 1];
            acc -= ya[r] * wb[c] + ya[r + NA] * wb[c + NA] + ya[r + 2 * NA] * wb[c + 2 * NA];
        }
        sblk[(size_t)NA * NA * bk + l] = acc;
    } else if (j == k && l < NA * NA + NA) {
        const int r = l - NA * NA;
        double acc = 0.0;
        for (int s = s0; s < s1; s++) acc += t[(size_t)NA * term[2 * s] + r];
        rhs[(size_t)NA * j + r] = (owner ? eA[(size_t)NA * j + r] : 0.0) - acc;
    }
}

// -------------------------------------------------------------------------
// Schur groups: one workgroup per group of consecutive chunks (<= BA_CH_OBS
// observations of consecutive points each).  Software-pipelined: while chunk
// k is being reduced, chunk k+1's W rows, V / eB and metadata record (one
// contiguous blob) are in flight into registers.  Per chunk:
//   V*^-1 per point (bundle_euclid.m:168-180; written for the back substitution)
//   Y = W V*^-1 in LDS (:182, never stored)
//   block sums: lane (chunk slot, row half, column pair) sums the chunk's terms
//     (points ascending) and adds them to the group accumulator of the block
//   e_ sums per camera: t_o = Y_o eB_i (mex_bundle_2_Se_.c:143-147)
// Accumulation order per entry: chunks ascending, terms ascending ->
// deterministic.  A "direct" group (one chunk touching more blocks than the LDS
// accumulators hold) writes its sums straight to HBM.
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(256) void k_schur_group(
    const int *__restrict__ grp_ch, const int *__restrict__ grp_gs,
    const int *__restrict__ grp_ge, const int *__restrict__ ch_pt,
    const int *__restrict__ ch_obase, const int *__restrict__ ch_blob,
    const unsigned *__restrict__ blob, const double *__restrict__ V,
    const double *__restrict__ eB, const double *__restrict__ W, double lambda, int bcap,
    int gcap, int ecap, double *__restrict__ Vinv, double *__restrict__ spart,
    double *__restrict__ epart)
{
    constexpr int WS = 3 * NA;
    constexpr int NR = (NA + 1) / 2;          // rows per half
    constexpr int NCP = (NA + 1) / 2;         // column pairs
    constexpr int IT = 2 * NCP;               // lanes per slot
    constexpr int GS_CAP = BA_GACC / (NA * NA);
    constexpr int WREG = (BA_CH_OBS * WS + 255) / 256;
    constexpr int BREG = 4;                   // blob words per lane in registers
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *Wl = sm;                                 // [CH_OBS][WS]
    double *Yl = Wl + BA_CH_OBS * WS;                // [CH_OBS][WS]
    double *Vl = Yl + BA_CH_OBS * WS;                // [CH_PTS][9]  V*^-1
    double *El = Vl + BA_CH_PTS * 9;                 // [CH_PTS][3]
    double *gacc = El + BA_CH_PTS * 3;               // [gcap][NA*NA]
    double *geacc = gacc + gcap * NA * NA;           // [ecap][NA]
    unsigned *bl = (unsigned *)(geacc + ecap * NA);  // [bcap] metadata record
    __shared__ int gp0[BA_GROUP_CH + 1], gob[BA_GROUP_CH + 1], gbo[BA_GROUP_CH + 1];
    const int g = blockIdx.x, tid = threadIdx.x;
    const int c0 = grp_ch[g], nc = grp_ch[g + 1] - c0;
    const int gs0 = grp_gs[g], ngs = grp_gs[g + 1] - gs0;
    const int ge0 = grp_ge[g], nge = grp_ge[g + 1] - ge0;
    const bool direct = ngs > GS_CAP;
    STAMP_DECL;
    if (!direct) {
        for (int q = tid; q < ngs * NA * NA; q += 256) gacc[q] = 0.0;
        for (int q = tid; q < nge * NA; q += 256) geacc[q] = 0.0;
    }
    for (int q = tid; q <= nc; q += 256) {
        gp0[q] = ch_pt[c0 + q];
        gob[q] = ch_obase[c0 + q];
        gbo[q] = ch_blob[c0 + q];
    }
    __syncthreads();
    double wreg[WREG], vreg[9], ereg[3];
    unsigned breg[BREG];
    // unconditional loads from clamped addresses: a load under a lane
    // condition becomes a branch + vmcnt(0) per element (cdna_hip_programming.md)
    auto fetch = [&](int k) {
        const int ob = gob[k], nw = (gob[k + 1] - ob) * WS;
        const double *src = W + (size_t)WS * ob;
        const int wl = nw > 0 ? nw - 1 : 0;
        if (nw == 0) src = W;
#pragma unroll
        for (int u = 0; u < WREG; u++) wreg[u] = src[min(tid + 256 * u, wl)];
        const int i0 = gp0[k], np = gp0[k + 1] - i0;
        const size_t i = (size_t)i0 + (np > 0 ? min(tid, np - 1) : 0);
        const double *vs = np > 0 ? V + 9 * i : V;
        const double *es = np > 0 ? eB + 3 * i : eB;
#pragma unroll
        for (int q = 0; q < 9; q++) vreg[q] = vs[q];
#pragma unroll
        for (int q = 0; q < 3; q++) ereg[q] = es[q];
        const unsigned *bs = blob + gbo[k];
        const int bl1 = gbo[k + 1] - gbo[k] - 1;   // a record is never empty
#pragma unroll
        for (int u = 0; u < BREG; u++) breg[u] = bs[min(tid + 256 * u, bl1)];
    };
    fetch(0);
    STAMP(0);
    for (int k = 0; k < nc; k++) {
        const int p0 = gp0[k], np = gp0[k + 1] - p0;
        const int obase = gob[k], nobs = gob[k + 1] - obase;
        const int nbw = gbo[k + 1] - gbo[k];
        // stage chunk k from registers
#pragma unroll
        for (int u = 0; u < WREG; u++) {
            const int q = tid + 256 * u;
            if (q < nobs * WS) Wl[q] = wreg[u];
        }
#pragma unroll
        for (int u = 0; u < BREG; u++) {
            const int q = tid + 256 * u;
            if (q < nbw) bl[q] = breg[u];
        }
        for (int q = tid + 256 * BREG; q < nbw; q += 256) bl[q] = blob[gbo[k] + q];
        if (tid < np) {   // V* -> V*^-1 from this lane's own registers
            const int i = p0 + tid;
            double vs[9], vi[9];
#pragma unroll
            for (int q = 0; q < 9; q++) vs[q] = vreg[q];
#pragma unroll
            for (int c = 0; c < 3; c++) vs[4 * c] = (1 + lambda) * vs[4 * c];
            vlg_pinv3(vs, vi);
#pragma unroll
            for (int q = 0; q < 9; q++) {
                Vl[9 * tid + q] = vi[q];
                Vinv[9 * (size_t)i + q] = vi[q];
            }
#pragma unroll
            for (int q = 0; q < 3; q++) El[3 * tid + q] = ereg[q];
        }
        __syncthreads();
        STAMP(1);
        if (k + 1 < nc) fetch(k + 1);   // in flight during the work below
        const unsigned h1 = bl[1];
        const int ns = (int)(h1 & 0xffffu), nes = (int)(h1 >> 16), nt = (int)bl[2];
        const unsigned *soff = bl + 4;
        const unsigned *eoff = soff + ns + 1;
        const unsigned *sgl = eoff + nes + 1;
        const unsigned *egl = sgl + ns;
        const unsigned *lpt = egl + nes;
        const unsigned *terml = lpt + nobs;
        const unsigned *eobl = terml + nt;
        // Y = W V*^-1 (bundle_euclid.m:182): lane (obs, row) forms the row's 3 entries
        for (int q = tid; q < nobs * NA; q += 256) {
            const int lo = q / NA, r = q % NA;
            const double *w = Wl + WS * lo;
            const double *vi = Vl + 9 * lpt[lo];
            const double w0 = w[r], w1 = w[r + NA], w2 = w[r + 2 * NA];
            double *y = Yl + WS * lo + r;
#pragma unroll
            for (int c = 0; c < 3; c++)
                y[NA * c] = fma(w2, vi[2 + 3 * c], fma(w1, vi[1 + 3 * c], w0 * vi[3 * c]));
        }
        __syncthreads();
        STAMP(2);
        // block sums over the chunk's terms: lane (slot, row half, column pair,
        // term parity); the two parities are combined by a lane shuffle
        for (int q = tid; q < ns * IT * 2; q += 256) {
            const int par = q & 1, qq = q >> 1;
            const int s = qq / IT, rh = (qq % IT) / NCP, c0c = 2 * (qq % NCP);
            const int r0 = rh * NR, nr = (rh == 0) ? NR : NA - NR;
            const bool two = c0c + 1 < NA;
            const int c1c = two ? c0c + 1 : c0c;
            double acc0[NR], acc1[NR];
#pragma unroll
            for (int r = 0; r < NR; r++) acc0[r] = acc1[r] = 0.0;
            const int u1 = (int)soff[s + 1];
            for (int u = (int)soff[s] + par; u < u1; u += 2) {
                const unsigned tw = terml[u];
                const double *y = Yl + WS * (tw & 0xffffu) + r0;
                const double *w = Wl + WS * (tw >> 16);
                const double wa0 = w[c0c], wa1 = w[c0c + NA], wa2 = w[c0c + 2 * NA];
                const double wb0 = w[c1c], wb1 = w[c1c + NA], wb2 = w[c1c + 2 * NA];
#pragma unroll
                for (int r = 0; r < NR; r++) {
                    if (r < nr) {
                        const double y0 = y[r], y1 = y[r + NA], y2 = y[r + 2 * NA];
                        acc0[r] = fma(y2, wa2, fma(y1, wa1, fma(y0, wa0, acc0[r])));
                        acc1[r] = fma(y2, wb2, fma(y1, wb1, fma(y0, wb0, acc1[r])));
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < NR; r++) {
                acc0[r] += __shfl_xor(acc0[r], 1, 64);
                acc1[r] += __shfl_xor(acc1[r], 1, 64);
            }
            if (par) continue;
            double *dst = direct ? spart + (size_t)NA * NA * (gs0 + s)
                                 : gacc + NA * NA * sgl[s];
#pragma unroll
            for (int r = 0; r < NR; r++) {
                if (r < nr) {
                    double *d0 = dst + (r0 + r) + NA * c0c;
                    *d0 = direct ? acc0[r] : *d0 + acc0[r];
                    if (two) {
                        double *d1 = dst + (r0 + r) + NA * (c0c + 1);
                        *d1 = direct ? acc1[r] : *d1 + acc1[r];
                    }
                }
            }
        }
        // e_ sums: t_o = Y_o eB_i (mex_bundle_2_Se_.c:143-147) summed per camera,
        // on the lanes the block sums leave idle (highest thread ids first)
        for (int q = 255 - tid; q < nes * NA; q += 256) {
            const int s = q / NA, r = q % NA;
            double acc = 0.0;
            const int u1 = (int)eoff[s + 1];
            for (int u = (int)eoff[s]; u < u1; u++) {
                const int lo = (int)eobl[u];
                const double *y = Yl + WS * lo;
                const double *eb = El + 3 * lpt[lo];
                acc = fma(y[r + 2 * NA], eb[2], fma(y[r + NA], eb[1], fma(y[r], eb[0], acc)));
            }
            if (direct) epart[(size_t)NA * (ge0 + s) + r] = acc;
            else geacc[NA * egl[s] + r] += acc;
        }
        STAMP(3);
        __syncthreads();
        STAMP(4);
    }
    if (!direct) {
        for (int q = tid; q < ngs * NA * NA; q += 256) spart[(size_t)NA * NA * gs0 + q] = gacc[q];
        for (int q = tid; q < nge * NA; q += 256) epart[(size_t)NA * ge0 + q] = geacc[q];
    }
    STAMP(5);
    if (tid == 0) {
#ifdef BA_STAMPS
        atomicAdd(&g_stamp[6], (unsigned long long)nc);
        atomicAdd(&g_stamp[7], 1ull);
#endif
    }
}

// -------------------------------------------------------------------------
// V*^-1 per point (bundle_euclid.m:168-180) for the MFMA Schur path
// -------------------------------------------------------------------------
// (the block's 256 contiguous 9-double rows in and out through LDS, lane by
// lane: every cache line requested once)
template <int NA>
__global__ __launch_bounds__(256) void k_point_vinv(const double *__restrict__ V, int n,
                                                    double lambda, double *__restrict__ Vinv)
{
    __shared__ double vsh[256 * 9];
    const int i0 = blockIdx.x * 256, tid = threadIdx.x;
    const int cnt = 9 * min(256, n - i0);
    const double *src = V + 9 * (size_t)i0;
    double t[9];
#pragma unroll
    for (int u = 0; u < 9; u++) t[u] = tid + 256 * u < cnt ? src[tid + 256 * u] : 0.0;
#pragma unroll
    for (int u = 0; u < 9; u++) vsh[tid + 256 * u] = t[u];
    __syncthreads();
    if (i0 + tid < n) {
        double vs[9], vi[9];
#pragma unroll
        for (int q = 0; q < 9; q++) vs[q] = vsh[9 * tid + q];
#pragma unroll
        for (int c = 0; c < 3; c++) vs[4 * c] = (1 + lambda) * vs[4 * c];
        vlg_pinv3(vs, vi);
#pragma unroll
        for (int q = 0; q < 9; q++) vsh[9 * tid + q] = vi[q];
    }
    __syncthreads();
    double *dst = Vinv + 9 * (size_t)i0;
#pragma unroll
    for (int u = 0; u < 9; u++)
        if (tid + 256 * u < cnt) dst[tid + 256 * u] = vsh[tid + 256 * u];
}

// -------------------------------------------------------------------------
// Schur complement on fp64 MFMA, operands register-resident (default fast
// path when every track fits).  A chunk holds <= BA_MF_PTS = 4 x 5 consecutive
// points seeing <= BA_MF_CMAX cameras; wave w owns the chunk's points
// 5w .. 5w + 4.  With the dense chunk slabs
//     Wk[k][NA cs + r] = W_o[r][q],   Yk[k][NA cs + r] = Y_o[r][q],
// Y_o = W_o V*^-1_p (bundle_euclid.m:182; o = observation of point p in camera
// slot cs, cameras ascending; zero where p does not see cs), the wave's 16 K
// rows k = (point, component) are laid out per 4-row MFMA K step s and lane
// quarter lk (li = l & 15, lk = l >> 4) as
//     s = 0, 1, 2 : point 5w + lk, component q = s
//     s = 3       : point 5w + 4,  component q = lk  (lk = 3: zero row)
// so that for s < 3 a lane holds all three components of ITS point: it forms
//     Yk[(lk, s)][16 t + li] = sum_u Wk[(lk, u)][16 t + li] V*^-1[u][s]
// on the VALU from its own W fragments, and for s = 3 one MFMA per column tile
// (A = V*^-1 of point 5w + 4 in rows 0..2, B = its W fragment) leaves Y in
// register 0 in exactly the A-fragment layout.  Then
//     S(ti, tj) += sum_s mfma(Yk frag s ti, Wk frag s tj)   (lower tiles)
// (v_mfma_f64_16x16x4f64: A lane = [li][lk], B lane = [lk][li], C row =
// lk + 4 reg, col = li), i.e.
//     S_chunk[NA cs_j + r][NA cs_k + c] = sum_i Y_ij[r] . W_ik[c]
// over the chunk's points (mex_bundle_2_Se_.c:80-118; the pairs a point does
// not see add exact zeros); e_ partials sum_k Yk[k][.] eB[k] (:132-155).
// Y costs 3 MFMAs per chunk and wave (12 when it was D Wk on the matrix pipe).
// Consecutive chunks with one camera list (a run of video-like tracks) keep
// accumulating in the registers; at a change of cameras ("flush") the four
// waves add their sums of each lower entry of each co-visible block to the
// group accumulator in LDS in wave order.  Every sum runs in a fixed order ->
// deterministic run to run; only the grouping differs from the term kernel.
// -------------------------------------------------------------------------
#define BA_MF_KB 5   // points per K-block (one wave)
#ifndef BA_MF_ROW4
#define BA_MF_ROW4 1
#endif
// lane (lk, 4 b + i) <- lane (lk, 4 rg + i) within each 16-lane row (ds_swizzle
// bit mask mode on 32-lane halves: and 0x13 keeps bit 4 and the row i, or sets
// the row group)
template <int RG> __device__ __forceinline__ double row4_bcast_c(double v)
{
    constexpr int pat = 0x13 | ((RG << 2) << 5);
    const long long u = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)(u & 0xffffffffLL), pat);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(u >> 32), pat);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double row4_bcast(double v, int rg)
{
    switch (rg) {
    case 0: return row4_bcast_c<0>(v);
    case 1: return row4_bcast_c<1>(v);
    case 2: return row4_bcast_c<2>(v);
    default: return row4_bcast_c<3>(v);
    }
}
#ifndef BA_MF_PIPE
#define BA_MF_PIPE 0
#endif
// BA_MF_GATHER: the 16 lanes of a row need the same V*^-1 and eB entries (the
// row's point), so each row loads them once -- lane li one entry -- and the
// chunk's processing broadcasts them (DPP row_newbcast): one load per lane
// instead of ten, a fifth of the kernel's vector-memory data traffic (TD
// busy 78 %, profiles/r06/pmc_cfg3_summary.csv), and 18 fewer VGPRs held
// per chunk in flight.  The same values: bit-identical.
#ifndef BA_MF_GATHER
#define BA_MF_GATHER 1
#endif
// lane Q's value to every lane of its 16-lane row (v_mov_b64 DPP row_newbcast)
template <int Q> __device__ __forceinline__ double row16_bcast_c(double v)
{
    const long long u = __builtin_bit_cast(long long, v);
    const long long r = __builtin_amdgcn_mov_dpp(u, 0x150 + Q, 0xf, 0xf, true);   // v_mov_b64_dpp
    return __builtin_bit_cast(double, r);
}
#ifndef BA_MF_WAVES
#define BA_MF_WAVES 3
#endif
template <int NA>
__global__ __launch_bounds__(256, (NA == 6) ? BA_MF_WAVES : 1) void k_schur_mfma(
    const int *__restrict__ grp_ch, const int *__restrict__ grp_gs,
    const int *__restrict__ grp_ge, const int *__restrict__ ch_pt,
    const int *__restrict__ ch_obase, const int *__restrict__ ch_blob,
    const unsigned *__restrict__ blob, const double *__restrict__ W,
    const double *__restrict__ Vinv, const double *__restrict__ eB, int nobs_all, int n_all,
    int gcap, int ecap, double *__restrict__ spart, double *__restrict__ epart, int ngrp,
    ba_camred cred)
{
    // workgroups past the groups: the camera reduction of a relinearised pass
    // (independent of the Schur sums, due before k_schur_reduce), filling the
    // CUs the groups' tail leaves idle -- no side stream, no fork / join
    if ((int)blockIdx.x >= ngrp) {
        camera_reduce_wg<NA>((int)blockIdx.x - ngrp, cred);
        return;
    }
    constexpr int WS = 3 * NA;
    constexpr int RT = BA_MF_RT(NA);
    constexpr int NTL = RT * (RT + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *gacc = sm;                                   // [gcap][NA*NA]
    double *geacc = gacc + gcap * NA * NA;               // [ecap][NA]
    unsigned *rec = (unsigned *)(geacc + ecap * NA);     // the group's chunk records
    __shared__ int gp0[BA_GROUP_CH + 1], gob[BA_GROUP_CH + 1], gbo[BA_GROUP_CH + 1];
    // groups last to first: linearisation wrote W first to last (streamed past
    // the caches), so the W rows read here last are the first ones, still in
    // the Infinity Cache when k_point_update_chunk reads W first to last
    const int g = ngrp - 1 - (int)blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int c0 = grp_ch[g], nc = grp_ch[g + 1] - c0;
    const int gs0 = grp_gs[g], ngs = grp_gs[g + 1] - gs0;
    const int ge0 = grp_ge[g], nge = grp_ge[g + 1] - ge0;
    const int rb0 = ch_blob[c0], nrw = ch_blob[c0 + nc] - rb0;
    for (int q = tid; q < ngs * NA * NA; q += 256) gacc[q] = 0.0;
    for (int q = tid; q < nge * NA; q += 256) geacc[q] = 0.0;
    for (int q = tid; q < nrw; q += 256) rec[q] = blob[rb0 + q];
    for (int q = tid; q <= nc; q += 256) {
        gp0[q] = ch_pt[c0 + q];
        gob[q] = ch_obase[c0 + q];
        gbo[q] = ch_blob[c0 + q] - rb0;
    }
    __syncthreads();
    // lane constants: K rows of its fragments, slab columns of its tiles
    int ccs[RT], crr[RT];
#pragma unroll
    for (int t = 0; t < RT; t++) {
        ccs[t] = (16 * t + li) / NA;
        crr[t] = (16 * t + li) % NA;
    }
    // fragments of one chunk, unconditional loads from clamped addresses
    // Absent entries read the exact zeros of the row past the end of W / V*^-1 /
    // eB (no select after a load: its wait lands at the MFMA that consumes it);
    // addresses are a uniform chunk base plus a 32-bit lane offset.
    // vf: V*^-1 of point 5w + lk, entries (0,0) (1,0) (2,0) (1,1) (2,1) (2,2)
    // (symmetric); vf[6]: the s = 3 Y MFMA's A fragment V*^-1[lk][li] of point
    // 5w + 4 (zero outside rows li < 3, K lk < 3)
    auto load = [&](int k, double (&wf)[4][RT], double (&vf)[7], double (&ef)[4]) {
        // BA_MF_GATHER: vf[0] holds the row's gathered entry (lane li: V*^-1
        // entry li < 6, eB entry li - 6 < 3, eB of point 5 w + 4 for li >= 9),
        // vf[6] as before; the rest is formed by process()
        const unsigned *r = rec + gbo[k];
        const int np = gp0[k + 1] - gp0[k], i0 = gp0[k], ob = gob[k];
        const int C = (int)(r[1] & 0xffu);
        const unsigned char *tab = (const unsigned char *)(r + 2 + C + C * (C + 1) / 2);
        const double *wbase = W + (size_t)WS * ob;
        const double *vbase = Vinv + 9 * (size_t)i0;
        const double *ebase = eB + 3 * (size_t)i0;
        const int wz = WS * (nobs_all - ob), vz = 9 * (n_all - i0), ez = 3 * (n_all - i0);
        // one lane offset per (point, column tile) -- the zero row's when absent;
        // the components are immediate offsets from it (zero row: 3 NA doubles)
        const int pA = BA_MF_KB * wv + lk, p4 = BA_MF_KB * wv + 4;
        const bool pvA = pA < np, pv4 = lk < 3 && p4 < np;
#pragma unroll
        for (int t = 0; t < RT; t++) {
            const bool cvA = pvA && ccs[t] < C, cv4 = pv4 && ccs[t] < C;
            const int iA = tab[cvA ? pA * C + ccs[t] : 0];   // clamped read, no branch
            const int i4 = tab[cv4 ? p4 * C + ccs[t] : 0];
            const int oA = (cvA && iA != 0xff ? WS * iA : wz) + crr[t];
            const int o4 = (cv4 && i4 != 0xff ? WS * i4 + NA * lk : wz) + crr[t];
#pragma unroll
            for (int s = 0; s < 3; s++) wf[s][t] = wbase[oA + NA * s];
            wf[3][t] = wbase[o4];
        }
        if (BA_MF_GATHER) {
            // V*^-1 entries (0,0) (1,0) (2,0) (1,1) (2,1) (2,2) -> lanes 0..5
            const int vo = li + (li >= 3 ? 1 : 0) + (li >= 5 ? 2 : 0);
            const double *src = li < 6   ? vbase + (pvA ? 9 * pA + vo : vz)
                                : li < 9 ? ebase + (pvA ? 3 * pA + li - 6 : ez)
                                         : ebase + (pv4 ? 3 * p4 + lk : ez);
            vf[0] = *src;
            const bool dv = p4 < np && li < 3 && lk < 3;
            vf[6] = vbase[dv ? 9 * p4 + lk + 3 * li : vz];
        } else {
            const int oe = pvA ? 3 * pA : ez;
#pragma unroll
            for (int s = 0; s < 3; s++) ef[s] = ebase[oe + s];
            ef[3] = ebase[pv4 ? 3 * p4 + lk : ez];
            const int ov = pvA ? 9 * pA : vz;
#pragma unroll
            for (int u = 0; u < 6; u++) {
                constexpr int off[6] = {0, 1, 2, 4, 5, 8};
                vf[u] = vbase[ov + off[u]];
            }
            const bool dv = p4 < np && li < 3 && lk < 3;
            vf[6] = vbase[dv ? 9 * p4 + lk + 3 * li : vz];
        }
    };
    d4 accS[NTL];
    double eacc[RT];
#pragma unroll
    for (int u = 0; u < NTL; u++) accS[u] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < RT; t++) eacc[t] = 0.0;
    // one chunk: Y tiles, e_ sums, lower S tiles; flush at a change of cameras
    auto process = [&](int k, const double (&wc)[4][RT], const double (&vg)[7],
                       const double (&eg)[4]) {
        double vc[7], ec[4];
        if (BA_MF_GATHER) {   // the row's entries from its lanes 0..9
            vc[0] = row16_bcast_c<0>(vg[0]);
            vc[1] = row16_bcast_c<1>(vg[0]);
            vc[2] = row16_bcast_c<2>(vg[0]);
            vc[3] = row16_bcast_c<3>(vg[0]);
            vc[4] = row16_bcast_c<4>(vg[0]);
            vc[5] = row16_bcast_c<5>(vg[0]);
            vc[6] = vg[6];
            ec[0] = row16_bcast_c<6>(vg[0]);
            ec[1] = row16_bcast_c<7>(vg[0]);
            ec[2] = row16_bcast_c<8>(vg[0]);
            ec[3] = row16_bcast_c<9>(vg[0]);
        } else {
#pragma unroll
            for (int u = 0; u < 7; u++) vc[u] = vg[u];
#pragma unroll
            for (int s = 0; s < 4; s++) ec[s] = eg[s];
        }
        const unsigned *r = rec + gbo[k];
        const unsigned h1 = r[1];
        const int C = (int)(h1 & 0xffu), fl = (int)((h1 >> 8) & 0xffu), Rc = NA * C;
        // row tile by row tile: one Y tile live at a time.  Every tile runs (tiles
        // past the chunk's columns multiply exact zeros): no branch between the
        // next chunk's loads and the MFMAs, so their waits stay precise
        // s = 3 first, all column tiles: point 5w + 4 on the matrix pipe
        // (register 0 = A fragment), in flight while the VALU forms the rest
        double y4[RT];
        if (BA_MF_ROW4) {
            // v_mfma_f64_4x4x4: block b = li >> 2 takes V*^-1 rows (li & 3) (the
            // A fragment's first block, swizzled to all four) against columns
            // 16 ti + li and leaves row lk, column 16 ti + li: register 0 of
            // the 16x16x4 form, at a sixth of its matrix-pipe time
            const double va = row4_bcast(vc[6], 0);
#pragma unroll
            for (int ti = 0; ti < RT; ti++)
                y4[ti] = __builtin_amdgcn_mfma_f64_4x4x4f64(va, wc[3][ti], 0.0, 0, 0, 0);
        } else {
#pragma unroll
            for (int ti = 0; ti < RT; ti++)
                y4[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(vc[6], wc[3][ti],
                                                              d4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0)[0];
        }
#pragma unroll
        for (int ti = 0; ti < RT; ti++) {
            {
                double y[4];
                y[3] = y4[ti];
                // s < 3: Y_o[r][s] = sum_u W_o[r][u] V*^-1[u][s], the lane's own point
                y[0] = fma(wc[2][ti], vc[2], fma(wc[1][ti], vc[1], wc[0][ti] * vc[0]));
                y[1] = fma(wc[2][ti], vc[4], fma(wc[1][ti], vc[3], wc[0][ti] * vc[1]));
                y[2] = fma(wc[2][ti], vc[5], fma(wc[1][ti], vc[4], wc[0][ti] * vc[2]));
                eacc[ti] = fma(y[3], ec[3], fma(y[2], ec[2], fma(y[1], ec[1],
                                                                 fma(y[0], ec[0], eacc[ti]))));
                if (BA_MF_ROW4 && NA == 6 && ti == RT - 1) {
                    // the last row tile holds NA C - 32 real rows (4 for the usual
                    // six-camera chunk): v_mfma_f64_4x4x4 per group of 4 rows
                    // (tools/ubench_mfma4x4.hip: a sixth of the 16x16x4 time).
                    // Its blocks b = li >> 2 take rows 4 rg + (li & 3) (the A
                    // operand swizzled within each 16-lane row) against columns
                    // 16 tj + li (the B fragment as is) and leave row 4 rg + lk,
                    // column 16 tj + li -- component rg of the 16x16 tile's
                    // accumulator, same lane: the flush below is unchanged
#pragma unroll
                    for (int rg = 0; rg < 4; rg++) {
                        if (16 * ti + 4 * rg >= Rc) continue;   // (uniform) rows past the chunk
#pragma unroll
                        for (int s = 0; s < 4; s++) {
                            const double ya = row4_bcast(y[s], rg);
#pragma unroll
                            for (int tj = 0; tj <= ti; tj++) {
                                d4 &t = accS[ti * (ti + 1) / 2 + tj];
                                t[rg] = __builtin_amdgcn_mfma_f64_4x4x4f64(ya, wc[s][tj], t[rg], 0,
                                                                           0, 0);
                            }
                        }
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < 4; s++) {   // K step outer: neighbours independent
#pragma unroll
                        for (int tj = 0; tj <= ti; tj++)
                            accS[ti * (ti + 1) / 2 + tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                                y[s], wc[s][tj], accS[ti * (ti + 1) / 2 + tj], 0, 0, 0);
                    }
                }
            }
        }
        if (fl & 2) {   // flush: wave by wave into the group accumulators
            const unsigned *ge = r + 2;
            const unsigned *pair = ge + C;
            double ecol[RT];
#pragma unroll
            for (int t = 0; t < RT; t++) {   // e_ column sums over the lane quarters
                const double v0 = __shfl(eacc[t], li, 64), v1 = __shfl(eacc[t], li + 16, 64);
                const double v2 = __shfl(eacc[t], li + 32, 64), v3 = __shfl(eacc[t], li + 48, 64);
                ecol[t] = ((v0 + v1) + v2) + v3;
                eacc[t] = 0.0;
            }
            for (int w = 0; w < 4; w++) {
                if (wv == w) {
#pragma unroll
                    for (int ti = 0; ti < RT; ti++)
#pragma unroll
                        for (int tj = 0; tj <= ti; tj++) {
                            const int col = 16 * tj + li;
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                const int rr = 16 * ti + lk + 4 * q;
                                if (rr < Rc && col < Rc && rr >= col) {
                                    const int cr = rr / NA, cc = col / NA;
                                    const unsigned gsl = pair[cr * (cr + 1) / 2 + cc];
                                    if (gsl != 0xffffffffu)
                                        gacc[gsl * (NA * NA) + (rr - NA * cr) +
                                             NA * (col - NA * cc)] +=
                                            accS[ti * (ti + 1) / 2 + tj][q];
                                }
                            }
                        }
                    if (lk == 0) {
#pragma unroll
                        for (int t = 0; t < RT; t++) {
                            const int col = 16 * t + li;
                            if (col < Rc) {
                                const int cs = col / NA;
                                geacc[ge[cs] * NA + col - NA * cs] += ecol[t];
                            }
                        }
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (int u = 0; u < NTL; u++) accS[u] = d4{0.0, 0.0, 0.0, 0.0};
        }
    };
    // two register sets, software pipelined: the next chunk's fragments are in
    // flight while this chunk's MFMAs run (no register copies between sets)
#if BA_MF_PIPE
    double wa[4][RT], da[7], ea[4], wb[4][RT], db[7], eb[4];
    load(0, wa, da, ea);
    for (int k = 0; k < nc; k += 2) {
        load(min(k + 1, nc - 1), wb, db, eb);   // unconditional: a clamped reload at the end
        process(k, wa, da, ea);
        if (k + 1 >= nc) break;
        load(min(k + 2, nc - 1), wa, da, ea);
        process(k + 1, wb, db, eb);
    }
#else
    double wa[4][RT], da[7], ea[4];
    for (int k = 0; k < nc; k++) {
        load(k, wa, da, ea);
        process(k, wa, da, ea);
    }
#endif
    __syncthreads();
    for (int q = tid; q < ngs * NA * NA; q += 256) spart[(size_t)NA * NA * gs0 + q] = gacc[q];
    for (int q = tid; q < nge * NA; q += 256) epart[(size_t)NA * ge0 + q] = geacc[q];
}

// S blocks and e_ from the chunk partials, in chunk order; then (long tracks)
// the terms Y_a W_b^T of every long track that sees both cameras of the block,
// in track order: wave 0 finds them by a binary search of each of camera j's
// long observations among camera k's (both lists ascending by track, staged
// in LDS), compacts the matches in order, and every entry's lane subtracts
// them -- the order and the expression of the former per-pair slots, so the
// blocks are the same bit for bit.
// k_schur_reduce's direct assembly (ba_dev::asm_direct): S == nullptr: none
struct ba_direct {
    double *S;
    long long lds;
    double *status;
};

struct ba_longs {
    const int *pair_ptr;                         // NULL: no long tracks
    const int2 *pair;                            // per block (j obs, k obs) in track order
    const double *ylong, *W;
    int L0;                                      // first long observation
};

// Setup (once per context, the structure does not change between passes):
// per block (j, k), the long tracks that see both cameras, in track order, as
// (long obs of camera j, long obs of camera k) pairs.  Wave 0 searches each of
// camera j's long observations in camera k's list (both ascending by track,
// staged in LDS) and compacts the matches in order.  fill = 0: count them
// into cnt[bk]; fill = 1: write them at pair[ptr[bk] ...].  Lists longer than
// the LDS stage are merged in global memory by lane 0.
__global__ __launch_bounds__(64) void k_long_pairs(const int *__restrict__ blk_jk, int nb,
                                                   const int *__restrict__ cam_lptr,
                                                   const int *__restrict__ cam_lobs,
                                                   const int *__restrict__ cam_ltrk, int fill,
                                                   int *__restrict__ cnt,
                                                   const int *__restrict__ ptr,
                                                   int2 *__restrict__ pair)
{
    __shared__ int la[BA_LCAM_LDS], lt[BA_LCAM_LDS], lb[BA_LCAM_LDS], ltb[BA_LCAM_LDS];
    const int bk = blockIdx.x, l = threadIdx.x;
    if (bk >= nb) return;
    const int j = blk_jk[2 * bk], k = blk_jk[2 * bk + 1];
    const int a0 = cam_lptr[j], na_ = cam_lptr[j + 1] - a0;
    const int b0 = cam_lptr[k], nb_ = cam_lptr[k + 1] - b0;
    int at = fill ? ptr[bk] : 0;
    if (na_ == 0 || nb_ == 0) {
        if (!fill && l == 0) cnt[bk] = 0;
        return;
    }
    if (na_ > BA_LCAM_LDS || nb_ > BA_LCAM_LDS) {   // rare: sequential merge
        if (l != 0) return;
        int p = 0, q = 0, c = 0;
        while (p < na_ && q < nb_) {
            const int tp = cam_ltrk[a0 + p], tq = cam_ltrk[b0 + q];
            if (tp < tq) {
                p++;
            } else if (tq < tp) {
                q++;
            } else {
                if (fill) pair[at + c] = int2{cam_lobs[a0 + p], cam_lobs[b0 + q]};
                c++;
                p++;
                q++;
            }
        }
        if (!fill) cnt[bk] = c;
        return;
    }
    for (int q = l; q < na_; q += 64) {
        la[q] = cam_lobs[a0 + q];
        lt[q] = cam_ltrk[a0 + q];
    }
    for (int q = l; q < nb_; q += 64) {
        lb[q] = cam_lobs[b0 + q];
        ltb[q] = cam_ltrk[b0 + q];
    }
    __syncthreads();
    int c = 0;
    for (int q0 = 0; q0 < na_; q0 += 64) {
        const int q = q0 + l;
        int pos = -1;
        if (q < na_) {
            const int t = lt[q];
            int lo = 0, hi = nb_;   // first entry with track >= t
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (ltb[mid] < t) lo = mid + 1;
                else hi = mid;
            }
            if (lo < nb_ && ltb[lo] == t) pos = lo;
        }
        const unsigned long long msk = __ballot(pos >= 0);
        if (fill && pos >= 0) pair[at + c + __popcll(msk & ((1ull << l) - 1ull))] = int2{la[q], lb[pos]};
        c += __popcll(msk);
    }
    if (!fill && l == 0) cnt[bk] = c;
}

template <int NA>
__global__ void k_schur_reduce(const int *__restrict__ blk_jk, const int *__restrict__ blk_sptr,
                               const int *__restrict__ blk_slots,
                               const int *__restrict__ cam_eptr,
                               const int *__restrict__ cam_eslots,
                               const double *__restrict__ spart,
                               const double *__restrict__ epart, const double *__restrict__ U,
                               const double *__restrict__ eA, int nb, double lambda, int owner,
                               double *__restrict__ sblk, double *__restrict__ rhs, ba_longs lg,
                               ba_direct dir)
{
    constexpr int NN = NA * NA, WS = 3 * NA;
    // the long-track batches' Y / W rows: dynamic LDS, sized by the launch only
    // when this launch takes the long tracks' pairs (lg.pair_ptr) -- static
    // arrays (14 KB) held 11 of these one-wave workgroups on a CU where the
    // wave slots allow more, so the ~6000 blocks of config 3 ran in 2+ rounds
    extern __shared__ double lds_dyn[];
    double *ys = lds_dyn, *ws = lds_dyn + BA_LMATCH_BATCH * WS;
    __shared__ int dzero[NA];
    __shared__ double erhs[NA];
    const int bk = blockIdx.x, l = threadIdx.x;
    if (bk >= nb) return;
    if (dir.S && bk == 0 && l == 0) {   // (k_assemble_tiles' reset, which does not run)
        dir.status[0] = 0.0;   // non-positive pivot
        dir.status[1] = 0.0;   // bounded hand-off spin gave up
    }
    const int j = blk_jk[2 * bk], k = blk_jk[2 * bk + 1];
    double acc = 0.0;
    if (l < NN) {
        const int r = l % NA, c = l / NA;
        if (j == k && owner) {
            const double u = U[(size_t)NN * j + r + NA * c];
            acc = (r == c) ? (1 + lambda) * u : u;
        }
        // 8 independent loads in flight, subtracted in slot order (same result)
        int q = blk_sptr[bk];
        const int qe = blk_sptr[bk + 1];
        for (; q + 8 <= qe; q += 8) {
            double v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = spart[(size_t)NN * blk_slots[q + t] + l];
#pragma unroll
            for (int t = 0; t < 8; t++) acc -= v[t];
        }
        for (; q < qe; q++) acc -= spart[(size_t)NN * blk_slots[q] + l];
    } else if (j == k && l < NN + NA) {
        const int r = l - NN;
        double e = owner ? eA[(size_t)NA * j + r] : 0.0;
        int q = cam_eptr[j];
        const int qe = cam_eptr[j + 1];
        for (; q + 8 <= qe; q += 8) {
            double v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = epart[(size_t)NA * cam_eslots[q + t] + r];
#pragma unroll
            for (int t = 0; t < 8; t++) e -= v[t];
        }
        for (; q < qe; q++) e -= epart[(size_t)NA * cam_eslots[q] + r];
        if (!dir.S) rhs[(size_t)NA * j + r] = e;
        else erhs[r] = e;   // (written below, after the diagonal's pinv rule)
    }
    if (lg.pair_ptr) {
        // the block's long-track terms in track order: the pairs' Y / W rows
        // staged in LDS a batch at a time by every lane (all loads in flight
        // at once), then each entry's lane subtracts the batch's terms in order
        const int p0 = lg.pair_ptr[bk], nm = lg.pair_ptr[bk + 1] - p0;
        for (int q0 = 0; q0 < nm; q0 += BA_LMATCH_BATCH) {
            const int nbt = min(BA_LMATCH_BATCH, nm - q0);
            for (int idx = l; idx < nbt * WS; idx += blockDim.x) {
                const int bt = idx / WS, e = idx - WS * bt;
                const int2 pr = lg.pair[p0 + q0 + bt];
                ys[idx] = lg.ylong[(size_t)WS * pr.x + e];
                ws[idx] = lg.W[(size_t)WS * (lg.L0 + pr.y) + e];
            }
            __syncthreads();
            if (l < NN) {
                const int r = l % NA, c = l / NA;
                for (int bt = 0; bt < nbt; bt++) {
                    const double *y = ys + WS * bt, *w = ws + WS * bt;
                    acc -= y[r] * w[c] + y[r + NA] * w[c + NA] + y[r + 2 * NA] * w[c + 2 * NA];
                }
            }
            __syncthreads();
        }
    }
    if (l < NN) sblk[(size_t)NN * bk + l] = acc;
    if (dir.S) {
        // k_assemble_tiles' work for this block: its lower entries into S, and
        // for a diagonal block the rule for an exactly-zero diagonal (unit
        // pivot, zero rhs: pinv semantics)
        const int r = l % NA, c = l / NA;
        if (l < NN && (j > k || r >= c)) {
            const long long row = (long long)NA * j + r, col = (long long)NA * k + c;
            const bool z = j == k && r == c && acc == 0.0;
            dir.S[row + dir.lds * col] = z ? 1.0 : acc;
            if (j == k && r == c) dzero[r] = z;
        }
        __syncthreads();
        if (j == k && l >= NN && l < NN + NA)
            rhs[(size_t)NA * j + (l - NN)] = dzero[l - NN] ? 0.0 : erhs[l - NN];
    }
}

// The long tracks' (obs, obs) terms of the co-visible blocks after
// k_schur_reduce has written their slot sums (it then skips its pair loop):
// four lanes per block, lane q a (NA+1)/2-row x (NA+1)/2-column quarter of
// S_jk, each entry of it taking the block's pairs in track order with
// k_schur_reduce's expression -- the same operations on the same values in the
// same order, so bit-identical.  A lane's Y / W rows come straight from
// global memory (no LDS staging, no barriers): 2 (NA+1)/2 x 3 values per pair
// for (NA+1)^2/4 entries, against six LDS reads per entry.  lblk: the blocks
// with pairs, most pairs first (the lanes of a wave loop about as long).
template <int NA>
__global__ __launch_bounds__(256) void k_schur_long_acc(const int *__restrict__ lblk, int nlb,
                                                        const int *__restrict__ pair_ptr,
                                                        const int2 *__restrict__ pair,
                                                        const double *__restrict__ ylong,
                                                        const double *__restrict__ W, int L0,
                                                        double *__restrict__ sblk)
{
    constexpr int WS = 3 * NA, NN = NA * NA, RH = (NA + 1) / 2;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int li = t >> 2, q = t & 3;
    if (li >= nlb) return;
    const int bk = lblk[li];
    const int r0 = (q & 1) ? RH : 0, nr = (q & 1) ? NA - RH : RH;
    const int c0 = (q & 2) ? RH : 0, nc = (q & 2) ? NA - RH : RH;
    double *sb = sblk + (size_t)NN * bk;
    double acc[RH][RH];
#pragma unroll
    for (int i = 0; i < RH; i++)
#pragma unroll
        for (int j = 0; j < RH; j++)
            acc[i][j] = (i < nr && j < nc) ? sb[(r0 + i) + NA * (c0 + j)] : 0.0;
    // LA_U pairs per round, all their loads in flight before the first
    // subtraction (a round costs one memory latency, not LA_U); the next
    // round's pair indices are fetched during this one.  Past the end a slot
    // re-reads the block's first pair and takes +0 instead (its term is then
    // +0 and acc - (+0) is acc bit for bit, -0 included): the subtractions are
    // unconditional, so the compiler cannot sink a slot's loads behind the
    // previous slot's arithmetic.
    constexpr int LA_U = 4;
    const int pb = pair_ptr[bk], np = pair_ptr[bk + 1] - pb;
    int2 nx[LA_U];
#pragma unroll
    for (int u = 0; u < LA_U; u++) nx[u] = pair[pb + (u < np ? u : 0)];
    for (int u0 = 0; u0 < np; u0 += LA_U) {
        double yv[LA_U][3][RH], wv[LA_U][3][RH];
#pragma unroll
        for (int u = 0; u < LA_U; u++) {
            const double *y = ylong + (size_t)WS * nx[u].x + r0;
            const double *w = W + (size_t)WS * ((size_t)L0 + nx[u].y) + c0;
            const bool ok = u0 + u < np;
#pragma unroll
            for (int m = 0; m < 3; m++)
#pragma unroll
                for (int i = 0; i < RH; i++) {
                    const double a = i < nr ? y[i + NA * m] : 0.0;
                    const double b = i < nc ? w[i + NA * m] : 0.0;
                    yv[u][m][i] = ok ? a : 0.0;
                    wv[u][m][i] = ok ? b : 0.0;
                }
        }
#pragma unroll
        for (int u = 0; u < LA_U; u++) {
            const int q = u0 + LA_U + u;
            nx[u] = pair[pb + (q < np ? q : 0)];
        }
#pragma unroll
        for (int u = 0; u < LA_U; u++) {
#pragma unroll
            for (int i = 0; i < RH; i++)
#pragma unroll
                for (int j = 0; j < RH; j++)
                    acc[i][j] -= yv[u][0][i] * wv[u][0][j] + yv[u][1][i] * wv[u][1][j] +
                                 yv[u][2][i] * wv[u][2][j];
        }
    }
#pragma unroll
    for (int i = 0; i < RH; i++)
#pragma unroll
        for (int j = 0; j < RH; j++)
            if (i < nr && j < nc) sb[(r0 + i) + NA * (c0 + j)] = acc[i][j];
}

// t_o = Y_o eB_i for given Y (stage-2 entry; k_damp_point forms it otherwise)
template <int NA>
__global__ void k_point_yeb(const int *__restrict__ pt_ptr, const double *__restrict__ Y,
                            const double *__restrict__ eB, int n, double *__restrict__ t)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double eb0 = eB[3 * (size_t)i], eb1 = eB[3 * (size_t)i + 1],
                 eb2 = eB[3 * (size_t)i + 2];
    for (int o = pt_ptr[i]; o < pt_ptr[i + 1]; o++) {
        const double *y = Y + (size_t)3 * NA * o;
#pragma unroll
        for (int r = 0; r < NA; r++)
            t[(size_t)NA * o + r] = y[r] * eb0 + y[r + NA] * eb1 + y[r + 2 * NA] * eb2;
    }
}

// -------------------------------------------------------------------------
// dense lower S from the blocks (off-diagonal blocks: j > k only)
// -------------------------------------------------------------------------
template <int NA>
__global__ void k_assemble(const int *__restrict__ blk_jk, const double *__restrict__ sblk,
                           int nb, long long lds, int lower_only, double *__restrict__ S)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long long)nb * NA * NA) return;
    const int bk = (int)(g / (NA * NA)), l = (int)(g % (NA * NA));
    const int j = blk_jk[2 * bk], k = blk_jk[2 * bk + 1];
    const int r = l % NA, c = l / NA;
    const long long row = NA * j + r, col = NA * k + c;
    if (lower_only && row < col) return;
    S[row + lds * col] = sblk[g];
}

// -------------------------------------------------------------------------
// camera update: a_new = a + da (mex_bundle_3_db_new.c:137-140), the rotation
// table of a_new (R(a_new), R(a_new + h e_k), R(a_new + 0): k_rotations' five,
// so an accepted step swaps it in and the next linearisation needs no
// rotation launch), and the camera part of dp'(lambda dp + g)
// (bundle_euclid.m:215-217), one partial per 64-lane workgroup.
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(320) void k_camera_update(
    const double *__restrict__ a, const double *__restrict__ da,
    const double *__restrict__ eA, int m, double lambda, double *__restrict__ a_new,
    double *__restrict__ rot_new, double *__restrict__ part)
{
    // 64 cameras per block; wave k < 5 builds rotation k of each camera's
    // table (the libm-exact sin / cos chains run side by side), wave 0 also
    // forms a_new and the camera part of dp'(lambda dp + g) (one wave's sum,
    // the order of the 64-camera partials)
    const int lane = threadIdx.x & 63, k = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane;
    double an[NA];
    double acc = 0.0;
    if (j < m) {
#pragma unroll
        for (int c = 0; c < NA; c++) {
            const double d = da[(size_t)NA * j + c];
            an[c] = a[(size_t)NA * j + c] + d;
            if (k == 0) {
                a_new[(size_t)NA * j + c] = an[c];
                acc += d * (lambda * d + eA[(size_t)NA * j + c]);
            }
        }
        if constexpr (NA != BA_PROJ_NA) rotation_k(an, k, rot_new + 45 * (size_t)j);
    }
    if (k == 0) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
        if (lane == 0) part[blockIdx.x] = acc;
    }
}

// -------------------------------------------------------------------------
// point update: db_i (da[0 .. ndb) per camera: ndb = 6 as the MEX file,
// App. A Q3, or NA for bundle_euclid_nomex.m:268-277), b_new, new
// projections of the point's observations, new SSE and the point part of
// dp'(lambda dp + g)
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(256) void k_point_update(
    const int *__restrict__ pt_ptr, const int *__restrict__ obs_cam,
    const double *__restrict__ obs_x, const double *__restrict__ K4,
    const double *__restrict__ W, const double *__restrict__ da,
    const double *__restrict__ eB, const double *__restrict__ Vinv,
    const double *__restrict__ b, const double *__restrict__ a_new,
    const double *__restrict__ rot_new, int n, int ndb, double lambda, double *__restrict__ db,
    double *__restrict__ b_new, double *__restrict__ part_sse, double *__restrict__ part_dpg,
    const unsigned char *__restrict__ obs_vis, double *__restrict__ xh_out)
{
    double sse = 0.0, dpg = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        double rhs[3] = {eB[3 * (size_t)i], eB[3 * (size_t)i + 1], eB[3 * (size_t)i + 2]};
        const int o0 = pt_ptr[i], o1 = pt_ptr[i + 1];
        for (int o = o0; o < o1; o++) {
            const double *w = W + (size_t)3 * NA * o;
            const double *d = da + (size_t)NA * obs_cam[o];
            double dl[NA];
#pragma unroll
            for (int k = 0; k < NA; k++) dl[k] = k < ndb ? d[k] : 0.0;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double *wr = w + NA * r;
                double t = wr[0] * dl[0] + wr[1] * dl[1] + wr[2] * dl[2] + wr[3] * dl[3] +
                           wr[4] * dl[4] + wr[5] * dl[5];
#pragma unroll
                for (int k = 6; k < NA; k++)   // nomex semantics only (ndb = NA)
                    if (k < ndb) t = t + wr[k] * dl[k];
                rhs[r] -= t;
            }
        }
        const double *vi = Vinv + 9 * (size_t)i;
        double bn[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double dbr = vi[r] * rhs[0] + vi[r + 3] * rhs[1] + vi[r + 6] * rhs[2];
            db[3 * (size_t)i + r] = dbr;
            bn[r] = b[3 * (size_t)i + r] + dbr;
            b_new[3 * (size_t)i + r] = bn[r];
            dpg += dbr * (lambda * dbr + eB[3 * (size_t)i + r]);
        }
        for (int o = o0; o < o1; o++) {
            if (obs_vis && !obs_vis[o]) continue;
            const int j = obs_cam[o];
            double an[NA], xh[2];
#pragma unroll
            for (int c = 0; c < NA; c++) an[c] = a_new[(size_t)NA * j + c];
            if constexpr (NA == BA_PROJ_NA) {   // mex_bundle_proj_3_db_new.c:160-165
                vlg_project_proj(an, bn, xh);
            } else {
                double k4[4], Kc[9], R[9];
#pragma unroll
                for (int c = 0; c < 4; c++) k4[c] = K4[4 * (size_t)j + c];
#pragma unroll
                for (int q = 0; q < 9; q++) R[q] = rot_new[45 * (size_t)j + q];
                vlg_calib(Kc, k4, an, NA - 6);
                vlg_project(Kc, R, an + 3, bn, xh);
            }
            const double d0 = obs_x[2 * (size_t)o] - xh[0];
            const double d1 = obs_x[2 * (size_t)o + 1] - xh[1];
            sse += d0 * d0 + d1 * d1;
            if (xh_out) {
                xh_out[2 * (size_t)o] = xh[0];
                xh_out[2 * (size_t)o + 1] = xh[1];
            }
        }
    }
    block_sum_to<256>(sse, part_sse + blockIdx.x);
    __syncthreads();
    block_sum_to<256>(dpg, part_dpg + blockIdx.x);
}

// -------------------------------------------------------------------------
// Fast-path update, one workgroup per Schur chunk (<= BA_CH_OBS observations
// of consecutive points; the same arithmetic as k_point_update, with
// coalesced, LDS-staged accesses instead of one lane walking a point's W):
//   lane (obs, r): t_o[r] = W_o(:, r)' da_j over da(1 .. ndb)   (:113-120)
//   lane per point: rhs = eB_i - t_o1 - t_o2 - ... (cameras ascending),
//                   db_i = V_inv_i rhs, b_new = b + db, dp'(lambda dp + g)
//   lane per obs:   new projection with a_new, b_new, new SSE     (:149-166)
// SSE / dpg partials per chunk, summed in chunk order by k_sum_parts.
// -------------------------------------------------------------------------
template <int NA>
__global__ __launch_bounds__(256) void k_point_update_chunk(
    const int *__restrict__ ch_pt, const int *__restrict__ ch_obase,
    const int *__restrict__ pt_ptr, const int *__restrict__ obs_cam,
    const unsigned char *__restrict__ obs_lpt, const double *__restrict__ obs_x,
    const double *__restrict__ K4, const double *__restrict__ W,
    const double *__restrict__ da, const double *__restrict__ eB,
    const double *__restrict__ Vinv, const double *__restrict__ b,
    const double *__restrict__ a_new, const double *__restrict__ rot_new, int ndb,
    double lambda, double *__restrict__ db, double *__restrict__ b_new,
    double *__restrict__ part_sse, double *__restrict__ part_dpg, int nch_reg,
    const int *__restrict__ seg_pt, const int *__restrict__ seg_long,
    const int *__restrict__ long_o0, const double *__restrict__ dpg_long)
{
    __shared__ double wl[BA_CH_OBS * 3 * NA];   // the chunk's W rows, then t_o
    __shared__ double bn[BA_CH_PTS * 3];
    __shared__ int lptr_raw[BA_CH_PTS];   // pt_ptr[p0 + t], t < np (wave 0: np <= 64)
    const int ch = blockIdx.x, tid = threadIdx.x;
    // segment chunk of a long track: db / b_new come from k_long_db (the sum
    // over all the track's observations); this chunk projects its part
    const bool seg = ch >= nch_reg;
    const int p0 = seg ? seg_pt[ch - nch_reg] : ch_pt[ch];
    const int np = seg ? 1 : ch_pt[ch + 1] - p0;
    const int obase = ch_obase[ch], nobs = ch_obase[ch + 1] - obase;
    if (seg) {
        double dpg = 0.0;
        if (tid < 3) bn[tid] = b_new[3 * (size_t)p0 + tid];
        if (tid == 0) {
            const int l = seg_long[ch - nch_reg];
            // once per track (written by k_long_db in this pass; a vector load,
            // as every word an earlier launch of the pass writes, ba_internal.h)
            if (obase == long_o0[l])
                dpg = __hip_atomic_load(dpg_long + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        double sse = 0.0;
        if (tid < nobs) {
            const int o = obase + tid, j = obs_cam[o];
            const double bl[3] = {bn[0], bn[1], bn[2]};
            double an[NA], xh[2];
#pragma unroll
            for (int c = 0; c < NA; c++) an[c] = a_new[(size_t)NA * j + c];
            if constexpr (NA == BA_PROJ_NA) {
                vlg_project_proj(an, bl, xh);
            } else {
                double k4[4], Kc[9], R[9];
#pragma unroll
                for (int c = 0; c < 4; c++) k4[c] = K4[4 * (size_t)j + c];
#pragma unroll
                for (int q = 0; q < 9; q++) R[q] = rot_new[45 * (size_t)j + q];
                vlg_calib(Kc, k4, an, NA - 6);
                vlg_project(Kc, R, an + 3, bl, xh);
            }
            const double d0 = obs_x[2 * (size_t)o] - xh[0];
            const double d1 = obs_x[2 * (size_t)o + 1] - xh[1];
            sse = d0 * d0 + d1 * d1;
        }
        block_sum_to<256>(sse, part_sse + ch);
        __syncthreads();
        block_sum_to<256>(dpg, part_dpg + ch);
        return;
    }
    // Load order = dependence depth: the chunk's W rows (HBM, the bulk) first,
    // the point offsets by LDS-DMA, the observations, then their da rows; no
    // load sits in a branch (the compiler would wait on it before the next)
    constexpr int MAXE = (BA_CH_OBS * 3 * NA + 255) / 256;
    const int ne = nobs * 3 * NA;
    double wr[MAXE];
    int oj = 0, opl = 0;
    double ox0 = 0.0, ox1 = 0.0, dl[NA];
    if (nobs > 0) {
        // the chunk's W rows are one contiguous range: read lane by lane (each
        // cache line requested once, not six times by 48-byte-strided lanes)
        const double *wsrc = W + (size_t)3 * NA * obase;
#pragma unroll
        for (int u = 0; u < MAXE; u++) {
            const int e = tid + 256 * u;
            wr[u] = __builtin_nontemporal_load(wsrc + (e < ne ? e : 0));   // W's last reader
        }
        static_assert(BA_CH_PTS <= 64, "one wave loads the point offsets");
        if (tid < 64)   // wave 0
            // (&lptr_raw[0], not the bare array: the builtin does not decay an
            // array argument and would read its first element as the address)
            __builtin_amdgcn_global_load_lds(pt_ptr + p0 + min(tid, np - 1), &lptr_raw[0], 4, 0,
                                             0);
        // observation lanes: camera, point slot, x and the da row (zero past
        // ndb); lanes past the chunk's observations read its last one
        const int o = obase + min(tid, nobs - 1);
        oj = obs_cam[o];
        opl = obs_lpt[o];
        ox0 = obs_x[2 * (size_t)o];
        ox1 = obs_x[2 * (size_t)o + 1];
        const double *d = da + (size_t)NA * oj;
#pragma unroll
        for (int k = 0; k < NA; k++) dl[k] = d[k];
#pragma unroll
        for (int k = 0; k < NA; k++)
            if (k >= ndb) dl[k] = 0.0;
#pragma unroll
        for (int u = 0; u < MAXE; u++) {
            const int e = tid + 256 * u;
            if (e < ne) wl[e] = wr[u];
        }
    }
    __syncthreads();
    // t_o[r] = W_o(:, r)' da_j, into the row's first slot (only this lane reads
    // the row)
    if (tid < nobs) {
        double *wo = wl + 3 * NA * tid;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            double *w = wo + NA * r;
            double t = w[0] * dl[0] + w[1] * dl[1] + w[2] * dl[2] + w[3] * dl[3] +
                       w[4] * dl[4] + w[5] * dl[5];
#pragma unroll
            for (int k = 6; k < NA; k++)   // nomex semantics only (ndb = NA)
                if (k < ndb) t = t + w[k] * dl[k];
            w[0] = t;
        }
    }
    __syncthreads();
    double dpg = 0.0, sse = 0.0;
    if (tid < np) {
        const int i = p0 + tid;
        double rhs[3] = {eB[3 * (size_t)i], eB[3 * (size_t)i + 1], eB[3 * (size_t)i + 2]};
        const int lo1 = tid + 1 < np ? lptr_raw[tid + 1] - obase : nobs;
        for (int lo = lptr_raw[tid] - obase; lo < lo1; lo++) {
#pragma unroll
            for (int r = 0; r < 3; r++) rhs[r] -= wl[3 * NA * lo + NA * r];
        }
        const double *vi = Vinv + 9 * (size_t)i;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double dbr = vi[r] * rhs[0] + vi[r + 3] * rhs[1] + vi[r + 6] * rhs[2];
            const double bnr = b[3 * (size_t)i + r] + dbr;
            db[3 * (size_t)i + r] = dbr;
            b_new[3 * (size_t)i + r] = bnr;
            bn[3 * tid + r] = bnr;
            dpg += dbr * (lambda * dbr + eB[3 * (size_t)i + r]);
        }
    }
    __syncthreads();
    if (tid < nobs) {
        const int j = oj, pl = opl;
        const double bl[3] = {bn[3 * pl], bn[3 * pl + 1], bn[3 * pl + 2]};
        double an[NA], xh[2];
#pragma unroll
        for (int c = 0; c < NA; c++) an[c] = a_new[(size_t)NA * j + c];
        if constexpr (NA == BA_PROJ_NA) {   // mex_bundle_proj_3_db_new.c:160-165
            vlg_project_proj(an, bl, xh);
        } else {
            double k4[4], Kc[9], R[9];
#pragma unroll
            for (int c = 0; c < 4; c++) k4[c] = K4[4 * (size_t)j + c];
#pragma unroll
            for (int q = 0; q < 9; q++) R[q] = rot_new[45 * (size_t)j + q];
            vlg_calib(Kc, k4, an, NA - 6);
            vlg_project(Kc, R, an + 3, bl, xh);
        }
        const double d0 = ox0 - xh[0];
        const double d1 = ox1 - xh[1];
        sse = d0 * d0 + d1 * d1;
    }
    block_sum_to<256>(sse, part_sse + ch);
    __syncthreads();
    block_sum_to<256>(dpg, part_dpg + ch);
}

// -------------------------------------------------------------------------
// Long tracks (more observations than a chunk holds; points [p_long, n) of the
// fast path).  Their observations are linearised by segment chunks of
// k_linearize_chunk; here:
//   k_long_vsum  : V_i, eB_i = the sum of the segments' partials (segment order)
//   k_long_y     : Y_a = W_a V*^-1 of every observation of the track (the block
//                  terms Y_a W_b^T, mex_bundle_2_Se_.c:80-118, are summed by
//                  k_schur_reduce) and Y_a eB_i (:132-155, one group e-slot
//                  per observation)
//   k_long_db    : db_i = V*^-1 (eB_i - sum_o W_o^T da_j) over all the track's
//                  observations (mex_bundle_3_db_new.c:99-134), b_new, dp'g
// -------------------------------------------------------------------------
__global__ void k_long_vsum(const int *__restrict__ long_pt, const int *__restrict__ long_seg0,
                            const double *__restrict__ vseg, double *__restrict__ V,
                            double *__restrict__ eB)
{
    const int l = blockIdx.x, e = threadIdx.x;
    if (e >= 12) return;
    const int i = long_pt[l];
    double acc = 0.0;
    for (int sg = long_seg0[l]; sg < long_seg0[l + 1]; sg++) acc += vseg[12 * (size_t)sg + e];
    if (e < 9) V[9 * (size_t)i + e] = acc;
    else eB[3 * (size_t)i + e - 9] = acc;
}

template <int NA>
__global__ __launch_bounds__(256) void k_long_y(const int *__restrict__ long_pt,
                                                const int *__restrict__ long_o0,
                                                const int *__restrict__ long_ebase,
                                                const double *__restrict__ W,
                                                const double *__restrict__ Vinv,
                                                const double *__restrict__ eB,
                                                double *__restrict__ ylong,
                                                double *__restrict__ epart)
{
    constexpr int WS = 3 * NA;
    const int tid = threadIdx.x, l = blockIdx.x;
    const int i = long_pt[l], o0 = long_o0[l], k = long_o0[l + 1] - o0, L0 = long_o0[0];
    double vi[9], eb[3];
#pragma unroll
    for (int q = 0; q < 9; q++) vi[q] = Vinv[9 * (size_t)i + q];
#pragma unroll
    for (int q = 0; q < 3; q++) eb[q] = eB[3 * (size_t)i + q];
    // Y_a = W_a V*^-1 (bundle_euclid.m:182; each entry summed left to right)
    for (int q = tid; q < k * WS; q += 256) {
        const int lo = q / WS, e = q - WS * lo, r = e % NA, c = e / NA;
        const double *w = W + (size_t)WS * (o0 + lo);
        ylong[(size_t)WS * (o0 - L0 + lo) + e] =
            w[r] * vi[3 * c] + w[r + NA] * vi[1 + 3 * c] + w[r + 2 * NA] * vi[2 + 3 * c];
    }
    // the e_ terms Y_a eB_i (mex_bundle_2_Se_.c:132-155): one group e-slot each
    const long long eb0 = long_ebase[l];
    for (int q = tid; q < k * NA; q += 256) {
        const int al = q / NA, r = q - NA * al;
        const double *w = W + (size_t)WS * (o0 + al);
        double y[3];
#pragma unroll
        for (int c = 0; c < 3; c++)
            y[c] = w[r] * vi[3 * c] + w[r + NA] * vi[1 + 3 * c] + w[r + 2 * NA] * vi[2 + 3 * c];
        epart[(size_t)NA * (eb0 + al) + r] = y[0] * eb[0] + y[1] * eb[1] + y[2] * eb[2];
    }
}

template <int NA>
__global__ __launch_bounds__(256) void k_long_db(
    const int *__restrict__ long_pt, const int *__restrict__ long_o0,
    const int *__restrict__ obs_cam, const double *__restrict__ W,
    const double *__restrict__ da, const double *__restrict__ eB,
    const double *__restrict__ Vinv, const double *__restrict__ b, int ndb, double lambda,
    double *__restrict__ db, double *__restrict__ b_new, double *__restrict__ dpg_long)
{
    __shared__ double red[3][256];
    const int l = blockIdx.x, tid = threadIdx.x;
    const int i = long_pt[l], o0 = long_o0[l], o1 = long_o0[l + 1];
    double t[3] = {0.0, 0.0, 0.0};
    for (int o = o0 + tid; o < o1; o += 256) {
        const double *d = da + (size_t)NA * obs_cam[o];
        double dl[NA];
#pragma unroll
        for (int kk = 0; kk < NA; kk++) dl[kk] = kk < ndb ? d[kk] : 0.0;
#pragma unroll
        for (int r = 0; r < 3; r++) {   // the expression of k_point_update_chunk
            const double *w = W + (size_t)3 * NA * o + NA * r;
            double v = w[0] * dl[0] + w[1] * dl[1] + w[2] * dl[2] + w[3] * dl[3] + w[4] * dl[4] +
                       w[5] * dl[5];
#pragma unroll
            for (int kk = 6; kk < NA; kk++)
                if (kk < ndb) v = v + w[kk] * dl[kk];
            t[r] += v;
        }
    }
#pragma unroll
    for (int r = 0; r < 3; r++) red[r][tid] = t[r];
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {   // fixed-order tree: deterministic
        if (tid < h)
            for (int r = 0; r < 3; r++) red[r][tid] += red[r][tid + h];
        __syncthreads();
    }
    if (tid == 0) {
        const double rhs[3] = {eB[3 * (size_t)i] - red[0][0], eB[3 * (size_t)i + 1] - red[1][0],
                               eB[3 * (size_t)i + 2] - red[2][0]};
        const double *vi = Vinv + 9 * (size_t)i;
        double dpg = 0.0;
        for (int r = 0; r < 3; r++) {
            const double dbr = vi[r] * rhs[0] + vi[r + 3] * rhs[1] + vi[r + 6] * rhs[2];
            db[3 * (size_t)i + r] = dbr;
            b_new[3 * (size_t)i + r] = b[3 * (size_t)i + r] + dbr;
            dpg += dbr * (lambda * dbr + eB[3 * (size_t)i + r]);
        }
        dpg_long[l] = dpg;
    }
}

// three fixed-order sums in one launch (block b: part[b] over n[b] -> out[b])
struct ba_sum3 {
    const double *part[3];
    int n[3];
    double *out[3];
    // optional publish (k_publish folded in): the last block to finish copies
    // scal[0..5] to the host-mapped hres, then the sequence number
    const double *scal;
    double *hres;
    double seq;
    unsigned *cnt;   // zero between launches (the last block resets it)
};

__global__ __launch_bounds__(1024) void k_sum_parts3(ba_sum3 a)
{
    const double *part = a.part[blockIdx.x];
    const int nparts = a.n[blockIdx.x];
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
    int q = threadIdx.x;
    for (; q + 3 * 1024 < nparts; q += 4 * 1024) {
        v0 += part[q];
        v1 += part[q + 1024];
        v2 += part[q + 2 * 1024];
        v3 += part[q + 3 * 1024];
    }
    for (; q < nparts; q += 1024) v0 += part[q];
    block_sum_to<1024>((v0 + v1) + (v2 + v3), a.out[blockIdx.x]);
    if (a.hres && threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(a.cnt, 1u) == 2u) {   // the three sums are in scal
            __threadfence();
            const volatile double *sc = a.scal;
            for (int k = 0; k < 6; k++) a.hres[k] = sc[k];
            __threadfence_system();
            *a.cnt = 0u;
            __atomic_store_n((unsigned long long *)(a.hres + 7), __double_as_longlong(a.seq),
                             __ATOMIC_RELEASE);
        }
    }
}

// fixed-order sum of nparts partials -> out (one 1024-thread block; four
// independent loads in flight per lane, so the latency of ~25 dependent
// rounds of HBM loads does not set the time)
#define BA_SUM_BS 1024
__global__ __launch_bounds__(BA_SUM_BS) void k_sum_parts(const double *__restrict__ part,
                                                         int nparts, double *__restrict__ out)
{
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
    int q = threadIdx.x;
    for (; q + 3 * BA_SUM_BS < nparts; q += 4 * BA_SUM_BS) {
        v0 += part[q];
        v1 += part[q + BA_SUM_BS];
        v2 += part[q + 2 * BA_SUM_BS];
        v3 += part[q + 3 * BA_SUM_BS];
    }
    for (; q < nparts; q += BA_SUM_BS) v0 += part[q];
    block_sum_to<BA_SUM_BS>((v0 + v1) + (v2 + v3), out);
}

// =========================================================================
// launchers
// =========================================================================
static inline int grid_for(long long work, int bs, int cap)
{
    long long g = (work + bs - 1) / bs;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

#define BA_DISPATCH(NAEXPR, CALL)                                                   \
    switch (NAEXPR) {                                                               \
    case 6: { constexpr int NA = 6; CALL; } break;                                  \
    case 7: { constexpr int NA = 7; CALL; } break;                                  \
    case 10: { constexpr int NA = 10; CALL; } break;                                \
    case BA_PROJ_NA: { constexpr int NA = BA_PROJ_NA; CALL; } break;                \
    default: return -1000;                                                          \
    }

static const int PT_GRID_CAP = 8192;  // partial-sum slots used by per-point kernels

int ba_launch_rotations(ba_dev *d, const double *a, double *rot, int all5)
{
    (void)all5;
    if (d->na == BA_PROJ_NA) return 0;   // projective camera: no rotations
    const int g = grid_for(d->m, 64, 1 << 30);
    KT_B(d);
    BA_DISPATCH(d->na, (k_rotations<NA><<<g, 64, 0, d->stream>>>(a, rot, d->m)));
    KT_E(d, KT_ROT);
    return -(int)hipGetLastError();
}

// the fast-path linearisation at (a, rot, b) into (W, V, eB, upart, chsse);
// u: the fused point update first (k_update_linearize)
template <int NA>
static void lin_chunk_launch(ba_dev *d, ba_flags f, const double *a, const double *rot,
                             const double *b, double *W, double *V, double *eB, double *upart,
                             double *chsse, const ba_upd *u)
{
    if (u)
        k_update_linearize<NA><<<d->nch, 256, 0, d->stream>>>(
            d->ch_pt, d->ch_obase, d->ch_eslot, d->eslot_optr, d->eslot_obs, d->pt_ptr,
            d->obs_cam, d->obs_lpt, d->obs_x, d->K4, a, rot, b, f, d->pivot, W, V, eB, upart,
            chsse, d->nch_reg, d->seg_pt, d->vseg, d->ch_cam, *u);
    else
        k_linearize_chunk<NA><<<d->nch, 256, 0, d->stream>>>(
            d->ch_pt, d->ch_obase, d->ch_eslot, d->eslot_optr, d->eslot_obs, d->pt_ptr,
            d->obs_cam, d->obs_lpt, d->obs_x, d->K4, a, rot, b, f, d->pivot, W, V, eB, upart,
            chsse, d->nch_reg, d->seg_pt, d->vseg, d->ch_cam);
}

int ba_launch_linearize(ba_dev *d, ba_flags f)
{
    if (!d->ordered) {
        KT_B(d);
        if (d->nch > 0)
            BA_DISPATCH(d->na, (lin_chunk_launch<NA>(d, f, d->a, d->rot, d->b, d->W, d->V,
                                                     d->eB, d->upart, d->chsse, nullptr)));
        if (d->nl > 0)   // long tracks: V / eB = sum of their segments' partials
            k_long_vsum<<<d->nl, 64, 0, d->stream>>>(d->long_pt, d->long_seg0, d->vseg, d->V,
                                                     d->eB);
        KT_E(d, KT_LIN);   // the SSE partials are summed by ba_launch_camera_reduce
        return -(int)hipGetLastError();
    }
    const int g = grid_for(d->n, 256, PT_GRID_CAP);
    KT_B(d);
    BA_DISPATCH(d->na, (k_linearize<NA><<<g, 256, 0, d->stream>>>(
                           d->pt_ptr, d->obs_cam, d->obs_x, d->K4, d->a, d->rot, d->b, d->n, f,
                           d->pivot, d->jrec, d->W, d->V, d->eB, d->part, d->xh_out,
                           d->B_out)));
    KT_E(d, KT_LIN);
    k_sum_parts<<<1, BA_SUM_BS, 0, d->stream>>>(d->part, g, d->scal + 0);
    return -(int)hipGetLastError();
}

int ba_launch_camera_reduce(ba_dev *d, ba_flags f, int fuse)
{
    const int bs = ((d->na * (d->na + 1) / 2 + d->na) + 63) / 64 * 64;
    if (!d->ordered) {
        // m camera workgroups + one for the SSE: scal[0] and the old_sse slot
        // after U | eA (all-reduced together with them)
        d->camred = ba_camred{d->cam_eptr, d->cam_eslots, d->upart, d->m, f, d->pivot,
                              d->U, d->eA, d->chsse, d->nch, d->scal + 0, d->eA + d->ld};
        if (fuse && d->ngrp_mf > 0 && d->fuse_camred) {   // run by this pass's MFMA Schur launch
            d->camred_pending = 1;
            return 0;
        }
        KT_B(d);
        BA_DISPATCH(d->na, (k_camera_reduce_chunks<NA><<<d->m + 1, 256, 0, d->stream>>>(
                               d->camred)));
        KT_E(d, KT_CAMRED);
        return -(int)hipGetLastError();
    }
    KT_B(d);
    BA_DISPATCH(d->na, (k_camera_reduce<NA><<<d->m, bs, 0, d->stream>>>(
                           d->cam_ptr, d->cam_obs, d->jrec, d->m, f, d->pivot, d->U, d->eA)));
    KT_E(d, KT_CAMRED);
    return -(int)hipGetLastError();
}

int ba_launch_damp_point(ba_dev *d, double lambda)
{
    const int g = grid_for(d->n, 256, PT_GRID_CAP);
    KT_B(d);
    BA_DISPATCH(d->na, (k_damp_point<NA><<<g, 256, 0, d->stream>>>(
                           d->pt_ptr, d->V, d->eB, d->W, d->n, lambda, d->Vinv, d->Y, d->t)));
    KT_E(d, KT_DAMP);
    return -(int)hipGetLastError();
}

int ba_launch_schur(ba_dev *d, double lambda)
{
    const int bs = ((d->na * d->na + d->na) + 63) / 64 * 64;
    KT_B(d);
    BA_DISPATCH(d->na, (k_schur<NA><<<d->nb, bs, 0, d->stream>>>(
                           d->blk_jk, d->blk_ptr, d->term, d->Y, d->W, d->t, d->U, d->eA, d->nb,
                           lambda, d->schur_owner, d->sblk, d->rhs)));
    KT_E(d, KT_SCHUR);
    return -(int)hipGetLastError();
}

#ifndef BA_SCHUR_TWO_STREAMS
#define BA_SCHUR_TWO_STREAMS 1
#endif
template <int NA>
static int launch_schur_fast(ba_dev *d, double lambda)
{
    // MFMA groups [0, ngrp_mf), then the per-term groups [ngrp_mf, ngrp)
    const bool two = BA_SCHUR_TWO_STREAMS && d->ngrp_mf > 0 && d->ngrp > d->ngrp_mf &&
                     !d->join_pending && d->side && !(d->kt && d->kt->on);
    if (d->ngrp_mf > 0) {
        KT_B(d);
        k_point_vinv<NA><<<(d->n + 255) / 256, 256, 0, d->stream>>>(d->V, d->n, lambda, d->Vinv);
        KT_E(d, KT_DAMP);
        if (two) VLGBA_CHECK(hipEventRecord(d->ev_fork, d->stream));   // V*^-1 ready
        const size_t sm2 = sizeof(double) * (d->mf_max_s * NA * NA + d->mf_max_e * NA) +
                           sizeof(unsigned) * (size_t)d->mf_max_blob;
        TRY_RC(ba_ensure_dyn_lds((const void *)k_schur_mfma<NA>, sm2));
        const int ncr = d->camred_pending ? d->m + 1 : 0;
        d->camred_pending = 0;
        KT_B(d);
        k_schur_mfma<NA><<<d->ngrp_mf + ncr, 256, sm2, d->stream>>>(
            d->grp_ch, d->grp_gs, d->grp_ge, d->ch_pt, d->ch_obase, d->ch_blob, d->blob, d->W,
            d->Vinv, d->eB, d->N, d->n, d->mf_max_s, d->mf_max_e, d->spart, d->epart,
            d->ngrp_mf, d->camred);
        KT_E(d, KT_SCHUR_MF);
    }
    if (d->ngrp > d->ngrp_mf) {
        const int gcap = d->grp_max_s, ecap = d->grp_max_e, bcap = d->max_blob;
        size_t smem = sizeof(double) * (2 * BA_CH_OBS * 3 * NA + BA_CH_PTS * 12 +
                                        gcap * NA * NA + ecap * NA) +
                      sizeof(unsigned) * bcap;
        smem = (smem + 15) & ~(size_t)15;
        TRY_RC(ba_ensure_dyn_lds((const void *)k_schur_group<NA>, smem));
        // beside the MFMA groups on the side stream (disjoint partial slots;
        // V*^-1 is ready): the two launches' tails overlap.  Untimed passes
        // only, and only when the side stream is idle (its camera reduction
        // ran inside k_schur_mfma); k_schur_reduce joins below.
        hipStream_t s0 = d->stream;
        if (two) {
            VLGBA_CHECK(hipStreamWaitEvent(d->side, d->ev_fork, 0));
            d->stream = d->side;
        }
        KT_B(d);
        k_schur_group<NA><<<d->ngrp - d->ngrp_mf, 256, smem, d->stream>>>(
            d->grp_ch + d->ngrp_mf, d->grp_gs + d->ngrp_mf, d->grp_ge + d->ngrp_mf, d->ch_pt,
            d->ch_obase, d->ch_blob, d->blob, d->V, d->eB, d->W, lambda, bcap, gcap, ecap,
            d->Vinv, d->spart, d->epart);
        KT_E(d, KT_SCHUR_CHUNK);
        if (two) {
            d->stream = s0;
            VLGBA_CHECK(hipEventRecord(d->ev_join, d->side));
            d->join_pending = 1;
        }
    }
    if (d->nl > 0) {   // long tracks: their V*^-1, then their (obs, obs) tiles
        KT_B(d);
        if (d->ngrp_mf == 0)   // (k_point_vinv above covered every point)
            k_point_vinv<NA><<<(d->n - d->p_long + 255) / 256, 256, 0, d->stream>>>(
                d->V + 9 * (size_t)d->p_long, d->n - d->p_long, lambda,
                d->Vinv + 9 * (size_t)d->p_long);
        k_long_y<NA><<<d->nl, 256, 0, d->stream>>>(d->long_pt, d->long_o0, d->long_ebase, d->W,
                                                   d->Vinv, d->eB, d->ylong, d->epart);
        KT_E(d, KT_SCHUR_CHUNK);
    }
    const int bs = ((NA * NA + NA) + 63) / 64 * 64;
    if (d->join_pending) {   // U / eA from the side stream's camera reduction
        VLGBA_CHECK(hipStreamWaitEvent(d->stream, d->ev_join, 0));
        d->join_pending = 0;
    }
    KT_B(d);
    ba_longs lg{};
    if (d->nl > 0 && !d->nlb) {
        lg.pair_ptr = d->lpair_ptr;
        lg.pair = d->lpair;
        lg.ylong = d->ylong;
        lg.W = d->W;
        lg.L0 = d->long_o0_h;
    }
    ba_direct dir{nullptr, 0, nullptr};
    if (d->asm_direct) dir = ba_direct{d->S, d->lds, d->scal + 4};
    const size_t lsh = lg.pair_ptr ? sizeof(double) * 2 * BA_LMATCH_BATCH * 3 * NA : 0;
    k_schur_reduce<NA><<<d->nb, bs, lsh, d->stream>>>(
        d->blk_jk, d->blk_gptr, d->blk_gslots, d->cam_gptr, d->cam_gslots, d->spart, d->epart,
        d->U, d->eA, d->nb, lambda, d->schur_owner, d->sblk, d->rhs, lg, dir);
    if (d->nl > 0 && d->nlb)   // the long tracks' terms after the slot sums
        k_schur_long_acc<NA><<<(4 * d->nlb + 255) / 256, 256, 0, d->stream>>>(
            d->lblk, d->nlb, d->lpair_ptr, d->lpair, d->ylong, d->W, d->long_o0_h, d->sblk);
    KT_E(d, KT_SCHUR_RED);
    return -(int)hipGetLastError();
}

int ba_launch_long_pairs(ba_dev *d, int fill, int *cnt)
{
    k_long_pairs<<<d->nb, 64, 0, d->stream>>>(d->blk_jk, d->nb, d->cam_lptr, d->cam_lobs,
                                              d->cam_ltrk, fill, cnt, d->lpair_ptr, d->lpair);
    return -(int)hipGetLastError();
}

int ba_launch_schur_fast(ba_dev *d, double lambda)
{
    switch (d->na) {
    case 6: return launch_schur_fast<6>(d, lambda);
    case 7: return launch_schur_fast<7>(d, lambda);
    case 10: return launch_schur_fast<10>(d, lambda);
    case BA_PROJ_NA: return launch_schur_fast<BA_PROJ_NA>(d, lambda);
    default: return -1000;
    }
}

// the pass's scalars to host-mapped memory, the sequence number after them
// (system-scope release): the host reads them without a copy or a stream sync
__global__ void k_publish(const double *__restrict__ scal, double *hres, double seq)
{
    if (threadIdx.x < 6) hres[threadIdx.x] = scal[threadIdx.x];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_store_n((unsigned long long *)(hres + 7), __double_as_longlong(seq),
                         __ATOMIC_RELEASE);
    }
}

int ba_launch_publish(ba_dev *d)
{
    d->seq++;
    k_publish<<<1, 64, 0, d->stream>>>(d->scal, d->hres_dev, (double)d->seq);
    return -(int)hipGetLastError();
}

int ba_launch_yeb(ba_dev *d)
{
    const int g = grid_for(d->n, 256, 1 << 30);
    BA_DISPATCH(d->na, (k_point_yeb<NA><<<g, 256, 0, d->stream>>>(d->pt_ptr, d->Y, d->eB, d->n,
                                                                    d->t)));
    return -(int)hipGetLastError();
}

int ba_launch_assemble(ba_dev *d)
{
    if (d->asm_direct) return 0;   // k_schur_reduce assembled S (ba_dev::asm_direct)
    KT_B(d);
    TRY_RC(ba_assemble_tiles(d));
    KT_E(d, KT_ASSEMBLE);
    return 0;
}

// The fused update (d->fused, fast path): k_camera_update, the long tracks'
// db, then ONE pass over the observations -- the point update and the
// linearisation at (a_new, b_new) into the second buffers (k_linearize_chunk
// with UPD: W2, V2, eB2, upart2, chsse2) -- and the pass's final sums: the new
// SSE is the sum of the new linearisation's per-chunk SSE partials.  lm_apply
// swaps the buffers when the step is accepted; a rejected step keeps the
// pass's own linearisation (App. A Q12).
static int launch_update_fused(ba_dev *d, double lambda, ba_flags f)
{
    const int gc = (d->m + 63) / 64;
    KT_B(d);
    const double lam_dpg = d->dpg_lambda ? lambda : 0.0;
    BA_DISPATCH(d->na, (k_camera_update<NA><<<gc, 320, 0, d->stream>>>(
                           d->a, d->da, d->eA, d->m, lam_dpg, d->a_new, d->rot_new,
                           d->part)));
    KT_E(d, KT_CAMUPD);
    KT_B(d);
    if (d->nl > 0)   // long tracks: db, b_new, dp'g over all their observations
        BA_DISPATCH(d->na, (k_long_db<NA><<<d->nl, 256, 0, d->stream>>>(
                               d->long_pt, d->long_o0, d->obs_cam, d->W, d->da, d->eB,
                               d->Vinv, d->b, d->ndb, lambda, d->db, d->b_new,
                               d->dpg_long)));
    const ba_upd u{d->W, d->da, d->eB, d->Vinv, d->b, d->ndb, lambda, d->db, d->b_new,
                   d->chsse2 + 2 * (size_t)d->nch, d->seg_long, d->long_o0, d->dpg_long};
    BA_DISPATCH(d->na, (lin_chunk_launch<NA>(d, f, d->a_new, d->rot_new, d->b_new, d->W2,
                                             d->V2, d->eB2, d->upart2, d->chsse2, &u)));
    if (d->nl > 0)   // long tracks: V2 / eB2 = sum of their segments' partials
        k_long_vsum<<<d->nl, 64, 0, d->stream>>>(d->long_pt, d->long_seg0, d->vseg, d->V2,
                                                 d->eB2);
    KT_E(d, KT_LIN_UPD);
    // new SSE (= the new linearisation's SSE), point dpg, camera dpg: one launch
    ba_sum3 s3 = {{d->chsse2, d->chsse2 + 2 * (size_t)d->nch, d->part},
                  {d->nch, d->nch, gc},
                  {d->scal + 1, d->scal + 3, d->scal + 2},
                  d->scal, nullptr, 0.0, d->pub_cnt};
    if (d->publish_req) {
        d->seq++;
        s3.hres = d->hres_dev;
        s3.seq = (double)d->seq;
        d->publish_req = 0;
        d->published = 1;
    }
    k_sum_parts3<<<3, 1024, 0, d->stream>>>(s3);
    return -(int)hipGetLastError();
}

int ba_launch_update(ba_dev *d, double lambda, ba_flags f)
{
    if (d->fused) return launch_update_fused(d, lambda, f);
    const int gc = (d->m + 63) / 64;
    KT_B(d);
    // lambda dp'dp once over the ranks (each adds da' eA of its partial eA)
    const double lam_dpg = d->dpg_lambda ? lambda : 0.0;
    BA_DISPATCH(d->na, (k_camera_update<NA><<<gc, 320, 0, d->stream>>>(
                           d->a, d->da, d->eA, d->m, lam_dpg, d->a_new, d->rot_new,
                           d->part)));
    KT_E(d, KT_CAMUPD);
    if (!d->ordered && d->nch > 0 && !d->obs_vis && !d->xh_out) {
        KT_B(d);
        if (d->nl > 0)   // long tracks: db, b_new, dp'g over all their observations
            BA_DISPATCH(d->na, (k_long_db<NA><<<d->nl, 256, 0, d->stream>>>(
                                   d->long_pt, d->long_o0, d->obs_cam, d->W, d->da, d->eB,
                                   d->Vinv, d->b, d->ndb, lambda, d->db, d->b_new,
                                   d->dpg_long)));
        BA_DISPATCH(d->na, (k_point_update_chunk<NA><<<d->nch, 256, 0, d->stream>>>(
                               d->ch_pt, d->ch_obase, d->pt_ptr, d->obs_cam, d->obs_lpt,
                               d->obs_x, d->K4, d->W, d->da, d->eB, d->Vinv, d->b, d->a_new,
                               d->rot_new, d->ndb, lambda, d->db, d->b_new, d->chsse + d->nch,
                               d->chsse + 2 * (size_t)d->nch, d->nch_reg, d->seg_pt,
                               d->seg_long, d->long_o0, d->dpg_long)));
        KT_E(d, KT_PTUPD);
        // new SSE, point dpg, camera dpg: one launch
        ba_sum3 s3 = {{d->chsse + d->nch, d->chsse + 2 * (size_t)d->nch, d->part},
                      {d->nch, d->nch, gc},
                      {d->scal + 1, d->scal + 3, d->scal + 2},
                      d->scal, nullptr, 0.0, d->pub_cnt};
        if (d->publish_req) {
            d->seq++;
            s3.hres = d->hres_dev;
            s3.seq = (double)d->seq;
            d->publish_req = 0;
            d->published = 1;
        }
        k_sum_parts3<<<3, 1024, 0, d->stream>>>(s3);
        return -(int)hipGetLastError();
    }
    k_sum_parts<<<1, BA_SUM_BS, 0, d->stream>>>(d->part, gc, d->scal + 2);
    const int g = grid_for(d->n, 256, PT_GRID_CAP);
    KT_B(d);
    BA_DISPATCH(d->na, (k_point_update<NA><<<g, 256, 0, d->stream>>>(
                           d->pt_ptr, d->obs_cam, d->obs_x, d->K4, d->W, d->da, d->eB, d->Vinv,
                           d->b, d->a_new, d->rot_new, d->n, d->ndb, lambda, d->db, d->b_new,
                           d->part + BA_PART_MAX, d->part + 2 * BA_PART_MAX, d->obs_vis,
                           d->xh_out)));
    KT_E(d, KT_PTUPD);
    k_sum_parts<<<1, BA_SUM_BS, 0, d->stream>>>(d->part + BA_PART_MAX, g, d->scal + 1);
    k_sum_parts<<<1, BA_SUM_BS, 0, d->stream>>>(d->part + 2 * BA_PART_MAX, g, d->scal + 3);
    return -(int)hipGetLastError();
}

// -------------------------------------------------------------------------
// Parity mode (vlgba_options.ordered = 2): the LM scalars summed sequentially
// in the reference's flat orders, by one lane, so that they equal the oracle's
// bit for bit:
//   e'e  over the dense 2 x n x m residual array in MATLAB's column-major
//        order (bundle_euclid.m:207-210: camera-major, points ascending, u then
//        v; the invisible entries are exact zeros and change nothing)
//   dp'(lambda dp + g) over dp = [da; db], g = [eA; eB] (:213-217)
// -------------------------------------------------------------------------
template <int NA>
__global__ void k_seq_old_sse(const int *__restrict__ cam_ptr, const int *__restrict__ cam_obs,
                              const double *__restrict__ jrec, int m, double *__restrict__ out)
{
    if (threadIdx.x != 0) return;
    constexpr int JS = 2 * NA + 2;
    double s = 0.0;
    for (int j = 0; j < m; j++)
        for (int q = cam_ptr[j]; q < cam_ptr[j + 1]; q++) {
            const double *e = jrec + (size_t)JS * cam_obs[q] + 2 * NA;
            s = s + e[0] * e[0];
            s = s + e[1] * e[1];
        }
    *out = s;
}

__global__ void k_seq_new_sums(const int *__restrict__ cam_ptr, const int *__restrict__ cam_obs,
                               const double *__restrict__ obs_x, const double *__restrict__ xh,
                               int m, const double *__restrict__ da,
                               const double *__restrict__ eA, long long ld,
                               const double *__restrict__ db, const double *__restrict__ eB,
                               int n, double lambda, double *__restrict__ scal)
{
    if (threadIdx.x != 0) return;
    double s = 0.0;
    for (int j = 0; j < m; j++)
        for (int q = cam_ptr[j]; q < cam_ptr[j + 1]; q++) {
            const int o = cam_obs[q];
            const double d0 = obs_x[2 * (size_t)o] - xh[2 * (size_t)o];
            const double d1 = obs_x[2 * (size_t)o + 1] - xh[2 * (size_t)o + 1];
            s = s + d0 * d0;
            s = s + d1 * d1;
        }
    double g = 0.0;
    for (long long k = 0; k < ld; k++) g = g + da[k] * (lambda * da[k] + eA[k]);
    for (long long k = 0; k < 3 * (long long)n; k++) g = g + db[k] * (lambda * db[k] + eB[k]);
    scal[1] = s;
    scal[2] = g;
    scal[3] = 0.0;
}

int ba_launch_parity_old_sse(ba_dev *d)
{
    BA_DISPATCH(d->na, (k_seq_old_sse<NA><<<1, 64, 0, d->stream>>>(d->cam_ptr, d->cam_obs,
                                                                   d->jrec, d->m, d->scal + 0)));
    return -(int)hipGetLastError();
}

int ba_launch_parity_new_sums(ba_dev *d, double lambda)
{
    k_seq_new_sums<<<1, 64, 0, d->stream>>>(d->cam_ptr, d->cam_obs, d->obs_x, d->xh_out, d->m,
                                            d->da, d->eA, d->ld, d->db, d->eB, d->n, lambda,
                                            d->scal);
    return -(int)hipGetLastError();
}

// dense (unpadded, both triangles) S for the stage-2 entry
int ba_launch_assemble_plain(ba_dev *d, double *S, long long ld, int lower_only)
{
    VLGBA_CHECK(hipMemsetAsync(S, 0, sizeof(double) * ld * ld, d->stream));
    const long long work = (long long)d->nb * d->na * d->na;
    const int g = (int)((work + 255) / 256);
    if (g > 0)
        BA_DISPATCH(d->na, (k_assemble<NA><<<g, 256, 0, d->stream>>>(d->blk_jk, d->sblk, d->nb,
                                                                       ld, lower_only, S)));
    return -(int)hipGetLastError();
}
