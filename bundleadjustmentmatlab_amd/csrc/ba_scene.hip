// ba_scene.hip -- synthetic banded scenes generated on the GPU (SURVEY.md
// sec. 8.f row 3: "GPU generation of 3M-obs scenes").
//
// The statistical model is the one of configs 2-4,
// itself a restatement of toolbox/test/generate_scene_and_motion.m:36-117
// (f = 500, c = (250, 250), 500 x 500 image, random-walk cameras, points at
// depth U(lo, hi) in front of their first camera, 0.5 px noise) with the
// perturbation of toolbox/test/demo_bundle_euclid.m:29-31 (w + 1e-3 N,
// T + 1e-4 N, X + 1e-3 N):
//   * cameras: damped random walk  vw = 0.8 vw + 2e-3 N,  vT = 0.8 vT + 2e-1 N
//   * point i: first camera s_i = floor((i + u_i) S / n), S = m - track + 1
//     (jittered strata: uniform marginal, points numbered in camera order as
//     generate_scene_and_motion.m:99-116 appends new features frame by frame),
//     pixel uv ~ U(image), depth d ~ U(lo, hi), X = R_s^T (d K^-1 [uv; 1] - T_s)
//   * observations: cameras s_i .. s_i + track - 1 (point-major, cameras
//     ascending), projection + noise N(0, noise^2) per coordinate
// Every random number has a fixed address in a counter-based generator
// (Philox4x32-10, key = seed; counter = (index, stream)), so the scene does not
// depend on the launch geometry, and tests/scene_ref.py restates it in numpy.
// Normals: Box-Muller on two 53-bit uniforms, the angle through the glibc
// sin / cos restatement (vlg_libm.h).
#include "vlgba.h"
#include "ba_internal.h"
#include "vlg_math.h"

#include <cstring>
#include <vector>

namespace {

struct u4 {
    unsigned x, y, z, w;
};

__device__ __forceinline__ u4 philox(unsigned long long idx, unsigned stream,
                                     unsigned long long seed)
{
    unsigned c0 = (unsigned)idx, c1 = (unsigned)(idx >> 32), c2 = stream, c3 = 0u;
    unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
        const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
        const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
        const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

// 53-bit uniform in [0, 1) from two words
__device__ __forceinline__ double unif(unsigned a, unsigned b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// two standard normals from one Philox block (Box-Muller)
__device__ __forceinline__ void normal2(u4 r, double &n0, double &n1)
{
    const double u1 = 1.0 - unif(r.x, r.y);   // (0, 1]
    const double u2 = unif(r.z, r.w);
    const double rad = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586 * u2;
    n0 = rad * vlg_lm_cos(th);
    n1 = rad * vlg_lm_sin(th);
}

enum { ST_CAM = 1, ST_PT = 2, ST_OBS = 3, ST_PCAM = 4, ST_PPT = 5 };

struct scene_dev {
    int m, n, track, S, keep_first_rotation;
    double f, cx, cy, width, height, dlo, dhi, noise;
    unsigned long long seed;
    double *K, *w, *T, *R, *X, *w0, *T0, *X0, *obs_x;
    int *start, *obs_pt, *obs_cam;
    unsigned *behind;   // per k_scene_obs block: observations behind their camera
};

// the walk's normals, one thread per camera (the transcendental part)
__global__ void k_scene_cam_noise(scene_dev s, double *nz)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < 1 || j >= s.m) return;
    for (int t = 0; t < 3; t++)
        normal2(philox(3ull * j + t, ST_CAM, s.seed), nz[6 * (size_t)j + 2 * t],
                nz[6 * (size_t)j + 2 * t + 1]);
}

// the camera walk: one lane, sequential over j (m steps of a few flops)
__global__ void k_scene_cams(scene_dev s, const double *nzall)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double vw[3] = {0.0, 0.0, 0.0}, vT[3] = {0.0, 0.0, 0.0};
    double w[3] = {0.0, 0.0, 0.0}, T[3] = {0.0, 0.0, 0.0};
    for (int j = 0; j < s.m; j++) {
        if (j > 0) {
            const double *nz = nzall + 6 * (size_t)j;
            for (int k = 0; k < 3; k++) {
                vw[k] = 0.8 * vw[k] + 2e-3 * nz[k];
                vT[k] = 0.8 * vT[k] + 2e-1 * nz[3 + k];
                w[k] = w[k] + vw[k];
                T[k] = T[k] + vT[k];
            }
        }
        for (int k = 0; k < 3; k++) {
            s.w[3 * (size_t)j + k] = w[k];
            s.T[3 * (size_t)j + k] = T[k];
        }
    }
}

// per camera: K, R (column major), the perturbed w0, T0
__global__ void k_scene_cam_par(scene_dev s)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= s.m) return;
    s.K[4 * (size_t)j] = s.f;
    s.K[4 * (size_t)j + 1] = s.f;
    s.K[4 * (size_t)j + 2] = s.cx;
    s.K[4 * (size_t)j + 3] = s.cy;
    double w[3] = {s.w[3 * (size_t)j], s.w[3 * (size_t)j + 1], s.w[3 * (size_t)j + 2]};
    double R[9];
    vlg_rodrigues(R, w);
    for (int q = 0; q < 9; q++) s.R[9 * (size_t)j + q] = R[q];
    double nz[6];
    for (int t = 0; t < 3; t++)
        normal2(philox(3ull * j + t, ST_PCAM, s.seed), nz[2 * t], nz[2 * t + 1]);
    for (int k = 0; k < 3; k++) {
        s.w0[3 * (size_t)j + k] =
            (s.keep_first_rotation && j == 0) ? w[k] : w[k] + nz[k] * 1e-3;
        s.T0[3 * (size_t)j + k] = s.T[3 * (size_t)j + k] + nz[3 + k] * 1e-4;
    }
}

// per point: first camera, world point, perturbed point
__global__ void k_scene_points(scene_dev s)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n) return;
    const u4 a = philox(2ull * i, ST_PT, s.seed), b = philox(2ull * i + 1, ST_PT, s.seed);
    const double uj = unif(a.x, a.y);
    int st = (int)(((double)i + uj) * (double)s.S / (double)s.n);
    st = st < s.S - 1 ? st : s.S - 1;
    const double u = unif(a.z, a.w) * s.width, v = unif(b.x, b.y) * s.height;
    const double d = s.dlo + (s.dhi - s.dlo) * unif(b.z, b.w);
    const double ray[3] = {(u - s.cx) / s.f * d, (v - s.cy) / s.f * d, 1.0 * d};
    const double *R = s.R + 9 * (size_t)st, *T = s.T + 3 * (size_t)st;
    double q[3] = {ray[0] - T[0], ray[1] - T[1], ray[2] - T[2]};
    double X[3];
    for (int r = 0; r < 3; r++)   // R^T q: column r of R (column major)
        X[r] = R[3 * r] * q[0] + R[3 * r + 1] * q[1] + R[3 * r + 2] * q[2];
    double nz[4];
    normal2(philox(2ull * i, ST_PPT, s.seed), nz[0], nz[1]);
    normal2(philox(2ull * i + 1, ST_PPT, s.seed), nz[2], nz[3]);
    s.start[i] = st;
    for (int r = 0; r < 3; r++) {
        s.X[4 * (size_t)i + r] = X[r];
        s.X0[4 * (size_t)i + r] = X[r] + nz[r] * 1e-3;
    }
    s.X[4 * (size_t)i + 3] = 1.0;
    s.X0[4 * (size_t)i + 3] = 1.0;
}

// per observation: camera, projection + noise
__global__ void k_scene_obs(scene_dev s)
{
    const long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long N = (long long)s.n * s.track;
    if (o >= N) return;
    const int i = (int)(o / s.track), j = s.start[i] + (int)(o - (long long)i * s.track);
    const double *R = s.R + 9 * (size_t)j, *T = s.T + 3 * (size_t)j, *X = s.X + 4 * (size_t)i;
    double Xc[3];
    for (int r = 0; r < 3; r++)
        Xc[r] = R[r] * X[0] + R[r + 3] * X[1] + R[r + 6] * X[2] + T[r];
    const double u = (s.f * Xc[0] + s.cx * Xc[2]) / Xc[2];
    const double v = (s.f * Xc[1] + s.cy * Xc[2]) / Xc[2];
    double n0, n1;
    normal2(philox((unsigned long long)o, ST_OBS, s.seed), n0, n1);
    s.obs_pt[o] = i;
    s.obs_cam[o] = j;
    s.obs_x[2 * o] = u + n0 * s.noise;
    s.obs_x[2 * o + 1] = v + n1 * s.noise;
}

// observations behind (or too close to) their camera, counted per block
__global__ void k_scene_check(scene_dev s)
{
    const long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long N = (long long)s.n * s.track;
    bool bad = false;
    if (o < N) {
        const int i = s.obs_pt[o], j = s.obs_cam[o];
        const double *R = s.R + 9 * (size_t)j, *T = s.T + 3 * (size_t)j, *X = s.X + 4 * (size_t)i;
        const double z = R[2] * X[0] + R[5] * X[1] + R[8] * X[2] + T[2];
        bad = !(z > 0.01 * s.dlo);
    }
    const int cnt = __syncthreads_count(bad);
    if (threadIdx.x == 0) s.behind[blockIdx.x] = (unsigned)cnt;
}

template <typename T>
int dalloc_t(T **p, size_t count)
{
    return hipMalloc((void **)p, sizeof(T) * (count ? count : 1)) == hipSuccess ? 0
                                                                                 : VLGBA_E_NOMEM;
}

}  // namespace

extern "C" int vlgba_scene_banded(const vlgba_scene_spec *sp, int device, vlgba_scene_out *out)
{
    if (!sp || !out || sp->m < 1 || sp->n < 0 || sp->track < 1) return VLGBA_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return VLGBA_E_ARG;
    scene_dev s;
    std::memset(&s, 0, sizeof s);
    s.m = sp->m;
    s.n = sp->n;
    s.track = sp->track < sp->m ? sp->track : sp->m;
    s.S = s.m - s.track + 1;
    s.keep_first_rotation = sp->keep_first_rotation;
    s.width = sp->width > 0 ? sp->width : 500.0;
    s.height = sp->height > 0 ? sp->height : 500.0;
    s.f = s.width;
    s.cx = s.width / 2;
    s.cy = s.height / 2;
    s.dlo = sp->depth_lo;
    s.dhi = sp->depth_hi;
    s.noise = sp->noise;
    s.seed = sp->seed;
    const long long N = (long long)s.n * s.track;
    if (N > 0x7fffffffLL) return VLGBA_E_ARG;
    if (out->num_obs_cap < N) return VLGBA_E_ARG;
    int rc = 0;
    hipStream_t st = nullptr;
    do {
        if ((rc = dalloc_t(&s.K, 4 * (size_t)s.m)) || (rc = dalloc_t(&s.w, 3 * (size_t)s.m)) ||
            (rc = dalloc_t(&s.T, 3 * (size_t)s.m)) || (rc = dalloc_t(&s.R, 9 * (size_t)s.m)) ||
            (rc = dalloc_t(&s.w0, 3 * (size_t)s.m)) || (rc = dalloc_t(&s.T0, 3 * (size_t)s.m)) ||
            (rc = dalloc_t(&s.X, 4 * (size_t)s.n)) || (rc = dalloc_t(&s.X0, 4 * (size_t)s.n)) ||
            (rc = dalloc_t(&s.start, (size_t)s.n)) || (rc = dalloc_t(&s.obs_pt, (size_t)N)) ||
            (rc = dalloc_t(&s.obs_cam, (size_t)N)) || (rc = dalloc_t(&s.obs_x, 2 * (size_t)N)) ||
            (rc = dalloc_t(&s.behind, (size_t)((N + 255) / 256))))
            break;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
            rc = -1;
            break;
        }
        const unsigned nblk = (unsigned)((N + 255) / 256);
        // the walk's normals in parallel, then the sequential recurrence (a
        // single lane evaluating 6m Box-Muller normals took ms)
        k_scene_cam_noise<<<(s.m + 63) / 64, 64, 0, st>>>(s, s.R);
        k_scene_cams<<<1, 64, 0, st>>>(s, s.R);
        k_scene_cam_par<<<(s.m + 63) / 64, 64, 0, st>>>(s);
        if (s.n > 0) {
            k_scene_points<<<(s.n + 255) / 256, 256, 0, st>>>(s);
            k_scene_obs<<<nblk, 256, 0, st>>>(s);
            k_scene_check<<<nblk, 256, 0, st>>>(s);
        }
        if (hipGetLastError() != hipSuccess) {
            rc = -1;
            break;
        }
        struct cp {
            void *dst;
            const void *src;
            size_t bytes;
        } cps[] = {{out->K, s.K, 32 * (size_t)s.m},      {out->w, s.w, 24 * (size_t)s.m},
                   {out->T, s.T, 24 * (size_t)s.m},      {out->w0, s.w0, 24 * (size_t)s.m},
                   {out->T0, s.T0, 24 * (size_t)s.m},    {out->X, s.X, 32 * (size_t)s.n},
                   {out->X0, s.X0, 32 * (size_t)s.n},    {out->obs_pt, s.obs_pt, 4 * (size_t)N},
                   {out->obs_cam, s.obs_cam, 4 * (size_t)N}, {out->obs_x, s.obs_x, 16 * (size_t)N}};
        for (const cp &c : cps)
            if (c.dst && c.bytes &&
                hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost, st) != hipSuccess)
                rc = -1;
        std::vector<unsigned> behind(nblk ? nblk : 1, 0u);
        if ((nblk && hipMemcpyAsync(behind.data(), s.behind, sizeof(unsigned) * nblk,
                                    hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = -1;
        if (!rc) {
            out->num_obs = N;
            out->behind = 0;
            for (unsigned b = 0; b < nblk; b++) out->behind += behind[b];
        }
    } while (0);
    if (st) (void)hipStreamSynchronize(st);
    for (void *p : {(void *)s.K, (void *)s.w, (void *)s.T, (void *)s.R, (void *)s.w0,
                    (void *)s.T0, (void *)s.X, (void *)s.X0, (void *)s.start, (void *)s.obs_pt,
                    (void *)s.obs_cam, (void *)s.obs_x, (void *)s.behind})
        if (p) (void)hipFree(p);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}
