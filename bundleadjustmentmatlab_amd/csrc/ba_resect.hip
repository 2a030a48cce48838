// ba_resect.hip -- batched one-camera bundle adjustment with the structure
// fixed: the non-linear refinement of estimate_camera.m:247-253,
//     [K T Omega] = bundle_euclid(K, T, Omega, X, x0, 'fix_calibration',
//                                 'fix_structure', 'visibility', inlier')
// (or without 'fix_calibration' for an uncalibrated camera), for many cameras
// at once (growing BA adds one camera per step and resects it; a whole batch of
// views can be resected against one structure).
//
// With m = 1 and 'fix_structure' the reference's pass (bundle_euclid.m:120-249)
// reduces exactly to: mex_bundle_1 for the camera's columns of A and e
// (mex_bundle_1_XABeUVWeAeB.c:192-256, 266-290, 317-323), the fix mask zeroing
// V, W, eB (bundle_euclid.m:140-144) so that V*^-1 = pinv(0) = 0, Y = 0,
// S = U* and e_ = eA - 0 (mex_bundle_2_Se_.c), da = pinv(S) e_ (:193), db = 0 and
// b unchanged (mex_bundle_3_db_new.c:99-146), the new projections, e'e and
// dp'(lambda dp + g) with the point entries exact zeros.  Every sum here runs
// sequentially in the reference's order (observations ascending) and the 6 x 6
// (num_a x num_a) solve is the parity-mode sequential Cholesky (pinv by cyclic
// Jacobi on a non-positive pivot), so each problem's trajectory equals the
// oracle's bundle_euclid restatement with m = 1 (vinv formula, solve / sums
// sequential) bit for bit.
//
// One workgroup per camera and LM pass: observations in tiles of 256 (one lane
// each: projection + num_a forward-difference columns into LDS), then
// NA*NA + NA + 1 accumulator lanes walk the tile in order.  The LM control
// (bundle_euclid.m:205-241, glibc pow for the lambda rule) stays on the host,
// per problem, exactly as vlgba_run applies it.
#include "ba_camera.h"
#include "../../include/vlgba.h"

#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#define RS_TILE 256

// state per problem: U (NA x NA) | eA (NA) | old SSE, kept across rejected
// passes (bundle_euclid.m:139 recomputes an identical linearisation, Q12)
template <int NA>
__global__ __launch_bounds__(256) void k_resect_pass(
    int nprob, const long long *__restrict__ obs_ptr, const double *__restrict__ Xw,
    const double *__restrict__ xo, const double *__restrict__ K4, double *__restrict__ a,
    double *__restrict__ a_new, double *__restrict__ state, const double *__restrict__ lam_p,
    const double *__restrict__ flags, double *__restrict__ out)
{
    constexpr int NUE = NA * NA + NA + 1;
    __shared__ double rot[45], rotn[9], k4[4], av[NA], an[NA];
    __shared__ double At[RS_TILE][2 * NA + 2];     // A (2 x NA, column major) | e
    __shared__ double st[NUE], S[NA * NA], rhs[NA], da[NA];
    __shared__ int fail;
    const int pb = blockIdx.x, tid = threadIdx.x;
    if (pb >= nprob) return;
    // staged with lambda as doubles (one copy a pass); a vector load at device
    // scope, as every per-pass word (ba_internal.h)
    const int fl = (int)__hip_atomic_load(flags + pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!(fl & 1)) return;                          // problem finished
    const long long o0 = obs_ptr[pb], no = obs_ptr[pb + 1] - o0;
    double *stg = state + (size_t)NUE * pb;
    if (tid < NA) {
        if (fl & 4) a[(size_t)NA * pb + tid] = a_new[(size_t)NA * pb + tid];   // accepted
    }
    if (tid < 4) k4[tid] = K4[4 * (size_t)pb + tid];
    __syncthreads();
    if (tid < NA) av[tid] = a[(size_t)NA * pb + tid];
    if (tid == 0) fail = 0;
    __syncthreads();
    if (fl & 2) {   // linearise at a (mex_bundle_1 for this camera)
        if (tid == 0) {
            const double w[3] = {av[0], av[1], av[2]};
            rotations5(w, rot);
        }
        double acc = 0.0;   // lane q < NUE: U[q] | eA[q - NA^2] | old SSE
        __syncthreads();
        const cam_view<NA> cv(av, k4, rot, 0);
        for (long long t0 = 0; t0 < no; t0 += RS_TILE) {
            const int nt = (int)(no - t0 < RS_TILE ? no - t0 : RS_TILE);
            if (tid < nt) {
                const long long o = o0 + t0 + tid;
                const double b[3] = {Xw[3 * o], Xw[3 * o + 1], Xw[3 * o + 2]};
                double xh[2];
                cv.project(b, xh);
                double *row = At[tid];
#pragma unroll 1
                for (int k = 0; k < NA; k++) {   // derivative_camera (:14-41)
                    double x1[2];
                    cv.project_dcam(k, b, x1);
                    row[2 * k] = vlg_fd_quot(x1[0] - xh[0]);
                    row[2 * k + 1] = vlg_fd_quot(x1[1] - xh[1]);
                }
                row[2 * NA] = xo[2 * o] - xh[0];          // e = X - X_hat (:222-223)
                row[2 * NA + 1] = xo[2 * o + 1] - xh[1];
            }
            __syncthreads();
            if (tid < NA * NA) {                  // U += A'A, entry (r, c) (:281-290)
                const int r = tid % NA, c = tid / NA;
                for (int q = 0; q < nt; q++)
                    acc += At[q][2 * r] * At[q][2 * c] + At[q][2 * r + 1] * At[q][2 * c + 1];
            } else if (tid < NA * NA + NA) {      // eA += A'e (:317-323)
                const int r = tid - NA * NA;
                for (int q = 0; q < nt; q++)
                    acc += At[q][2 * r] * At[q][2 * NA] + At[q][2 * r + 1] * At[q][2 * NA + 1];
            } else if (tid == NUE - 1) {          // e(:)'e(:) in MATLAB's flat order
                for (int q = 0; q < nt; q++) {
                    acc = acc + At[q][2 * NA] * At[q][2 * NA];
                    acc = acc + At[q][2 * NA + 1] * At[q][2 * NA + 1];
                }
            }
            __syncthreads();
        }
        if (tid < NUE) stg[tid] = acc;
    }
    __syncthreads();
    if (tid < NUE) st[tid] = stg[tid];
    __syncthreads();
    const double lambda = __hip_atomic_load(lam_p + pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
        // S = U* (damped diagonal), e_ = eA - 0: fix_structure zeroes V, W, eB,
        // so V*^-1 = pinv(0) = 0 and Y = 0 (bundle_euclid.m:140-193)
        for (int c = 0; c < NA; c++)
            for (int r = 0; r < NA; r++) {
                const double u = st[r + NA * c];
                S[r + NA * c] = (r == c) ? (1 + lambda) * u : u;
            }
        for (int r = 0; r < NA; r++) rhs[r] = st[NA * NA + r];
        // pinv rule for exactly-zero rows (App. A Q2 / Q8), then the sequential
        // Cholesky of the lower triangle (the parity-mode solve's loops)
        for (int j = 0; j < NA; j++)
            if (S[j + NA * j] == 0.0) {
                S[j + NA * j] = 1.0;
                rhs[j] = 0.0;
            }
        double L[NA * NA];
        for (int q = 0; q < NA * NA; q++) L[q] = S[q];
        bool ok = true;
        for (int j = 0; j < NA && ok; j++) {
            double s = L[j + NA * j];
            for (int k = 0; k < j; k++) s = s - L[j + NA * k] * L[j + NA * k];
            if (!(s > 0.0)) {
                ok = false;
                break;
            }
            const double p = sqrt(s);
            L[j + NA * j] = p;
            for (int i = j + 1; i < NA; i++) {
                double t = L[i + NA * j];
                for (int k = 0; k < j; k++) t = t - L[i + NA * k] * L[j + NA * k];
                L[i + NA * j] = t / p;
            }
        }
        if (ok) {
            double x[NA];
            for (int i = 0; i < NA; i++) {
                double t = rhs[i];
                for (int k = 0; k < i; k++) t = t - L[i + NA * k] * x[k];
                x[i] = t / L[i + NA * i];
            }
            for (int i = NA - 1; i >= 0; i--) {
                double t = x[i];
                for (int k = i + 1; k < NA; k++) t = t - L[k + NA * i] * x[k];
                x[i] = t / L[i + NA * i];
            }
            for (int i = 0; i < NA; i++) da[i] = x[i];
        } else {
            // da = pinv(S) e_ (bundle_euclid.m:193): cyclic Jacobi on the
            // symmetrised S, MATLAB's tolerance NA * eps(max |eigenvalue|)
            double A[NA][NA], Q[NA][NA];
            for (int p = 0; p < NA; p++)
                for (int q = 0; q < NA; q++) {
                    const double sp = p >= q ? S[p + NA * q] : S[q + NA * p];
                    A[p][q] = sp;
                    Q[p][q] = p == q ? 1.0 : 0.0;
                }
            for (int sweep = 0; sweep < 64; sweep++) {
                double off = 0.0;
                for (int p = 0; p < NA; p++)
                    for (int q = p + 1; q < NA; q++) off += A[p][q] * A[p][q];
                if (off == 0.0) break;
                for (int p = 0; p < NA - 1; p++)
                    for (int q = p + 1; q < NA; q++) {
                        if (A[p][q] == 0.0) continue;
                        const double th = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                        const double t = (th >= 0.0 ? 1.0 : -1.0) /
                                         (fabs(th) + sqrt(th * th + 1.0));
                        const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
                        for (int k = 0; k < NA; k++) {
                            const double u = A[k][p], v = A[k][q];
                            A[k][p] = c * u - sn * v;
                            A[k][q] = sn * u + c * v;
                        }
                        for (int k = 0; k < NA; k++) {
                            const double u = A[p][k], v = A[q][k];
                            A[p][k] = c * u - sn * v;
                            A[q][k] = sn * u + c * v;
                        }
                        for (int k = 0; k < NA; k++) {
                            const double u = Q[k][p], v = Q[k][q];
                            Q[k][p] = c * u - sn * v;
                            Q[k][q] = sn * u + c * v;
                        }
                    }
            }
            double emax = 0.0;
            for (int k = 0; k < NA; k++) emax = fmax(emax, fabs(A[k][k]));
            int e;
            (void)frexp(emax, &e);
            const double tol = emax > 0.0 ? NA * ldexp(1.0, e - 53) : 0.0;
            double x[NA] = {};
            for (int k = 0; k < NA; k++) {
                if (!(fabs(A[k][k]) > tol)) continue;
                double w = 0.0;
                for (int i = 0; i < NA; i++) w += Q[i][k] * rhs[i];
                w /= A[k][k];
                for (int i = 0; i < NA; i++) x[i] += Q[i][k] * w;
            }
            for (int i = 0; i < NA; i++) da[i] = x[i];
            fail = 1;
        }
    }
    __syncthreads();
    if (tid < NA) {   // a_new = a + da (mex_bundle_3_db_new.c:137-140)
        an[tid] = av[tid] + da[tid];
        a_new[(size_t)NA * pb + tid] = an[tid];
    }
    __syncthreads();
    if (tid == 0) {
        const double w[3] = {an[0], an[1], an[2]};
        vlg_rodrigues(rotn, w);
    }
    __syncthreads();
    // new projections (:149-166; b_new = b + db with db = 0), then e_new'e_new
    double nsum = 0.0;
    for (long long t0 = 0; t0 < no; t0 += RS_TILE) {
        const int nt = (int)(no - t0 < RS_TILE ? no - t0 : RS_TILE);
        if (tid < nt) {
            const long long o = o0 + t0 + tid;
            const double b[3] = {Xw[3 * o], Xw[3 * o + 1], Xw[3 * o + 2]};
            double Kc[9], xh[2];
            vlg_calib(Kc, k4, an, NA - 6);
            vlg_project(Kc, rotn, an + 3, b, xh);
            At[tid][0] = xo[2 * o] - xh[0];
            At[tid][1] = xo[2 * o + 1] - xh[1];
        }
        __syncthreads();
        if (tid == 0)
            for (int q = 0; q < nt; q++) {
                nsum = nsum + At[q][0] * At[q][0];
                nsum = nsum + At[q][1] * At[q][1];
            }
        __syncthreads();
    }
    if (tid == 0) {
        double g = 0.0;   // dp'(lambda dp + g): the point entries are exact zeros
        for (int k = 0; k < NA; k++) g = g + da[k] * (lambda * da[k] + st[NA * NA + k]);
        out[4 * (size_t)pb + 0] = st[NUE - 1];
        out[4 * (size_t)pb + 1] = nsum;
        out[4 * (size_t)pb + 2] = g;
        out[4 * (size_t)pb + 3] = fail ? 1.0 : 0.0;
    }
}

namespace {
template <typename T>
int dmalloc_n(T **p, size_t n)
{
    *p = (T *)ba_dmalloc(sizeof(T) * (n ? n : 1));
    return *p ? 0 : -(int)hipErrorOutOfMemory;
}
// Per-device pool of a stream and a pinned host block for the per-pass LM
// scalars: creating a stream and pageable copies cost more than the
// resection itself (the growing-BA replay calls it once per added camera).
struct rs_pool {
    int device;
    hipStream_t s;
    double *pin;     // pinned: lam [np] | flags [np] (as doubles) | out [4 np]
    size_t cap;      // doubles
};
std::mutex g_rs_pool_mu;
std::vector<rs_pool> g_rs_pool;

int rs_acquire(int device, size_t need, rs_pool &r)
{
    {
        std::lock_guard<std::mutex> lk(g_rs_pool_mu);
        for (size_t q = 0; q < g_rs_pool.size(); q++)
            if (g_rs_pool[q].device == device) {
                r = g_rs_pool[q];
                g_rs_pool.erase(g_rs_pool.begin() + (long)q);
                break;
            }
    }
    if (!r.s) {
        r.device = device;
        if (hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking) != hipSuccess) return -1;
    }
    if (r.cap < need) {
        if (r.pin) (void)hipHostFree(r.pin);
        r.pin = nullptr;
        r.cap = 0;
        const size_t cap = need > 4096 ? need : 4096;
        if (hipHostMalloc((void **)&r.pin, sizeof(double) * cap, hipHostMallocDefault) !=
            hipSuccess)
            return -1;
        r.cap = cap;
    }
    return 0;
}

void rs_release(const rs_pool &r)
{
    (void)hipStreamSynchronize(r.s);
    std::lock_guard<std::mutex> lk(g_rs_pool_mu);
    g_rs_pool.push_back(r);
}
}   // namespace

extern "C" int vlgba_resect(const vlgba_resect_problem *pr, const vlgba_options *opt, double *a,
                            double *error_out, int error_cap, int *num_error,
                            vlgba_stats *stats)
{
    if (!pr || !a || pr->nprob < 0 || !pr->obs_ptr || (error_out && error_cap < 0))
        return VLGBA_E_ARG;
    const int na = pr->num_a, np = pr->nprob;
    if (na != 6 && na != 7 && na != 10) return VLGBA_E_NUMA;
    if (np == 0) return 0;
    const long long N = pr->obs_ptr[np];
    if (pr->obs_ptr[0] != 0 || N < 0 || (N > 0 && (!pr->X || !pr->x)) || !pr->K)
        return VLGBA_E_ARG;
    for (int q = 0; q < np; q++)
        if (pr->obs_ptr[q + 1] < pr->obs_ptr[q]) return VLGBA_E_ARG;
    vlgba_options dflt;
    std::memset(&dflt, 0, sizeof dflt);
    if (!opt) opt = &dflt;
    const int max_iter = opt->max_iter > 0 ? opt->max_iter : 20;
    const int max_iter2 = opt->max_iter2 > 0 ? opt->max_iter2 : 10;
    const double lambda0 = opt->lambda0 > 0 ? opt->lambda0 : 1e-3;
    const double stop_rel = opt->stop_rel > 0 ? opt->stop_rel : 1e-3;
    VLGBA_CHECK(hipSetDevice(opt->device));
    const auto t0 = std::chrono::steady_clock::now();
    rs_pool pool{opt->device, nullptr, nullptr, 0};
    if (rs_acquire(opt->device, 6 * (size_t)np, pool)) {
        if (pool.s) rs_release(pool);
        return -1;
    }
    hipStream_t s = pool.s;
    double *h_lam = pool.pin, *h_fl = pool.pin + np, *h_out = pool.pin + 2 * (size_t)np;
    const int NUE = na * na + na + 1;
    long long *d_ptr = nullptr;
    double *d_X = nullptr, *d_x = nullptr, *d_K = nullptr, *d_a = nullptr, *d_an = nullptr;
    double *d_st = nullptr, *d_lam = nullptr, *d_out = nullptr, *d_fl = nullptr;
    int rc = 0;
    std::vector<double> lam(np, lambda0), nu(np, 2.0), out(4 * (size_t)np);
    std::vector<int> fl(np), iter(np, 1), iter2(np, 0), passes(np, 0), acc(np, 0);
    std::vector<std::vector<double>> err(np);
    std::vector<int> active(np, 1);
    int total_passes = 0, total_acc = 0;
    do {
        if ((rc = dmalloc_n(&d_ptr, np + 1)) || (rc = dmalloc_n(&d_X, 3 * (size_t)N)) ||
            (rc = dmalloc_n(&d_x, 2 * (size_t)N)) || (rc = dmalloc_n(&d_K, 4 * (size_t)np)) ||
            (rc = dmalloc_n(&d_a, (size_t)na * np)) || (rc = dmalloc_n(&d_an, (size_t)na * np)) ||
            (rc = dmalloc_n(&d_st, (size_t)NUE * np)) || (rc = dmalloc_n(&d_lam, 2 * (size_t)np)) ||
            (rc = dmalloc_n(&d_out, 4 * (size_t)np)))
            break;
        d_fl = d_lam + np;
        if (hipMemcpyAsync(d_ptr, pr->obs_ptr, sizeof(long long) * (np + 1), hipMemcpyHostToDevice,
                           s) != hipSuccess ||
            (N > 0 && (hipMemcpyAsync(d_X, pr->X, sizeof(double) * 3 * N, hipMemcpyHostToDevice,
                                      s) != hipSuccess ||
                       hipMemcpyAsync(d_x, pr->x, sizeof(double) * 2 * N, hipMemcpyHostToDevice,
                                      s) != hipSuccess)) ||
            hipMemcpyAsync(d_K, pr->K, sizeof(double) * 4 * np, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemcpyAsync(d_a, a, sizeof(double) * na * np, hipMemcpyHostToDevice, s) !=
                hipSuccess) {
            rc = -1;
            break;
        }
        std::vector<int> accepted_prev(np, 0), relin(np, 1);
        for (;;) {
            // bundle_euclid.m:120-123 per problem
            int nact = 0;
            for (int q = 0; q < np; q++) {
                if (!active[q]) continue;
                bool go = iter[q] < max_iter && iter2[q] < max_iter2;
                if (go && iter[q] >= 3) {
                    const double e1 = err[q][iter[q] - 1], e0 = err[q][iter[q] - 2];
                    go = e1 > 1e-20 && e0 - e1 > stop_rel * e0;
                }
                if (!go) active[q] = 0;
                nact += active[q];
                fl[q] = active[q] | (relin[q] ? 2 : 0) | (accepted_prev[q] ? 4 : 0);
            }
            if (!nact) break;
            for (int q = 0; q < np; q++) {   // pinned staging: one small copy per pass
                h_lam[q] = lam[q];
                h_fl[q] = (double)fl[q];
            }
            if (hipMemcpyAsync(d_lam, h_lam, sizeof(double) * 2 * np, hipMemcpyHostToDevice, s) !=
                hipSuccess) {
                rc = -1;
                break;
            }
            switch (na) {
            case 6:
                k_resect_pass<6><<<np, 256, 0, s>>>(np, d_ptr, d_X, d_x, d_K, d_a, d_an, d_st,
                                                    d_lam, d_fl, d_out);
                break;
            case 7:
                k_resect_pass<7><<<np, 256, 0, s>>>(np, d_ptr, d_X, d_x, d_K, d_a, d_an, d_st,
                                                    d_lam, d_fl, d_out);
                break;
            default:
                k_resect_pass<10><<<np, 256, 0, s>>>(np, d_ptr, d_X, d_x, d_K, d_a, d_an, d_st,
                                                     d_lam, d_fl, d_out);
                break;
            }
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(h_out, d_out, sizeof(double) * 4 * np, hipMemcpyDeviceToHost,
                               s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess) {
                rc = -1;
                break;
            }
            std::memcpy(out.data(), h_out, sizeof(double) * 4 * np);
            for (int q = 0; q < np; q++) {
                if (!active[q]) continue;   // a finished problem keeps its last flags
                accepted_prev[q] = 0;
                relin[q] = 0;
                const double old = out[4 * q], nw = out[4 * q + 1], dpg = out[4 * q + 2];
                const double num_vis = (double)(pr->obs_ptr[q + 1] - pr->obs_ptr[q]);
                const double rho = (old - nw) / dpg;
                passes[q]++;
                total_passes++;
                if ((old - nw) > 0) {   // bundle_euclid.m:218-232
                    const double olde = old / num_vis, newe = nw / num_vis;
                    if ((int)err[q].size() < iter[q]) err[q].push_back(olde);
                    else err[q][iter[q] - 1] = olde;
                    iter[q]++;
                    err[q].push_back(newe);
                    iter2[q] = 0;
                    lam[q] = lam[q] * std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3));
                    nu[q] = 2.0;
                    accepted_prev[q] = 1;
                    relin[q] = 1;
                    acc[q]++;
                    total_acc++;
                } else {                // :233-241
                    lam[q] = lam[q] * nu[q];
                    nu[q] = 2.0 * nu[q];
                    iter2[q]++;
                }
            }
        }
        if (rc) break;
        // the last accepted step's parameters
        for (int q = 0; q < np; q++) fl[q] = accepted_prev[q] ? 4 : 0;
        std::vector<double> an((size_t)na * np);
        if (hipMemcpyAsync(a, d_a, sizeof(double) * na * np, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipMemcpyAsync(an.data(), d_an, sizeof(double) * na * np, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = -1;
            break;
        }
        for (int q = 0; q < np; q++)
            if (accepted_prev[q])
                std::memcpy(a + (size_t)na * q, an.data() + (size_t)na * q, sizeof(double) * na);
        for (int q = 0; q < np; q++) {
            if (num_error) num_error[q] = (int)err[q].size();
            if (error_out)
                for (size_t k = 0; k < err[q].size() && k < (size_t)error_cap; k++)
                    error_out[(size_t)error_cap * q + k] = err[q][k];
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    for (void *p : {(void *)d_ptr, (void *)d_X, (void *)d_x, (void *)d_K, (void *)d_a,
                    (void *)d_an, (void *)d_st, (void *)d_lam, (void *)d_out})
        if (p) ba_dfree(p);
    rs_release(pool);
    if (stats) {
        stats->iterations = total_passes;
        stats->accepted = total_acc;
        stats->num_error = 0;
        stats->lambda = np ? lam[0] : 0.0;
        stats->pinv_passes = stats->spin_retries = stats->nd_retries = 0;
        stats->seconds =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}
