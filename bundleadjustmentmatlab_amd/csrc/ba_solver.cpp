// ba_solver.cpp -- libvlgba host side: problem setup, the LM driver of
// toolbox/bundle/bundle_euclid.m:111-249 and the C ABI of include/vlgba.h.
//
// The LM control flow stays on the host (it is a handful of scalars per pass,
// exactly as bundle_euclid.m keeps it in MATLAB); every array stays in HBM.
// One pass = rotations + linearize + camera reduce (skipped after a rejected
// step: bundle_euclid.m:139 recomputes an identical linearisation, App. A Q12)
// + damping/Y + Schur + dense Cholesky solve + update/new cost, then ONE
// device->host copy of 5 scalars.
//
// Multi-GPU (one process per GPU): points are split into
// contiguous ranges of balanced observation count; each rank linearises its
// points, RCCL all-reduces U/eA/old-SSE once per linearisation and the packed
// co-visible blocks of S + e_ once per pass, every rank runs the identical
// dense solve, and a 3-scalar all-reduce drives the accept/reject decision.
#include "ba_internal.h"
#include "../../include/vlgba.h"

#include <rccl/rccl.h>
#include <climits>
#include <rocsolver/rocsolver.h>   // types only: the library is dlopen'ed on first use

#include <dlfcn.h>
#include <unistd.h>
#include <cstdlib>
#include <string>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <map>
#include <new>
#include <numeric>
#include <thread>
#include <vector>

#define VLGBA_STR2(x) #x
#define VLGBA_STR(x) VLGBA_STR2(x)
#define VLGBA_VERSION_STR \
    "vlgba 0.2 (abi " VLGBA_STR(VLGBA_ABI_VERSION) ", gfx950, fp64, MFMA-f64 Cholesky)"

// ---------------------------------------------------------------------------
// Device memory: a per-device caching allocator.  A solve's context makes a few
// dozen allocations; hipMalloc / hipFree of each costs tens of microseconds,
// which the growing-BA replay (hundreds of small solves) would pay every time.
// Blocks are rounded up to a power of two (256 B .. 1 GiB) and kept on a free
// list when released; larger blocks go straight back to HIP.
// ---------------------------------------------------------------------------
namespace {
std::mutex g_mem_mu;
std::multimap<std::pair<int, size_t>, void *> g_mem_free;     // (device, bucket) -> block
std::unordered_map<void *, std::pair<int, size_t>> g_mem_live;  // block -> (device, bucket)
constexpr size_t BA_MEM_CACHE_MAX = size_t(1) << 30;

size_t mem_bucket(size_t bytes)
{
    if (bytes > BA_MEM_CACHE_MAX) return bytes;
    size_t b = 256;
    while (b < bytes) b <<= 1;
    return b;
}
}   // namespace

// VLGBA_POISON=1 (debugging): every block handed out is filled with 0xff
// bytes (NaN doubles, -1 ints), so a kernel that reads memory it never wrote
// shows up as NaN instead of as a stale value of a previous context
static void *poisoned(void *p, size_t b)
{
    static const bool on = std::getenv("VLGBA_POISON") != nullptr;
    if (on && p) {   // null-stream memset: not ordered with non-blocking streams
        (void)hipMemset(p, 0xff, b);
        (void)hipDeviceSynchronize();
    }
    return p;
}

void *ba_dmalloc(size_t bytes)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    const size_t b = mem_bucket(bytes ? bytes : 1);
    {
        std::lock_guard<std::mutex> lk(g_mem_mu);
        auto it = g_mem_free.find({dev, b});
        if (it != g_mem_free.end()) {
            void *p = it->second;
            g_mem_free.erase(it);
            g_mem_live[p] = {dev, b};
            return poisoned(p, b);
        }
    }
    void *p = nullptr;
    if (hipMalloc(&p, b) != hipSuccess) {
        // out of memory with blocks cached: give them back and retry once
        std::vector<void *> drop;
        {
            std::lock_guard<std::mutex> lk(g_mem_mu);
            for (auto &kv : g_mem_free) drop.push_back(kv.second);
            g_mem_free.clear();
        }
        for (void *q : drop) (void)hipFree(q);
        if (hipMalloc(&p, b) != hipSuccess) return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_mem_mu);
    g_mem_live[p] = {dev, b};
    return poisoned(p, b);
}

void ba_dfree(void *p)
{
    if (!p) return;
    std::unique_lock<std::mutex> lk(g_mem_mu);
    auto it = g_mem_live.find(p);
    if (it == g_mem_live.end()) {   // not ours
        lk.unlock();
        (void)hipFree(p);
        return;
    }
    const auto key = it->second;
    g_mem_live.erase(it);
    if (key.second > BA_MEM_CACHE_MAX) {
        lk.unlock();
        (void)hipFree(p);
        return;
    }
    g_mem_free.emplace(key, p);
}

int ba_ensure_dyn_lds(const void *fn, size_t bytes)
{
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, size_t> done;
    int dev = 0;
    VLGBA_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    size_t &have = done[{fn, dev}];
    if (bytes > have) {
        VLGBA_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)bytes));
        have = bytes;
    }
    return 0;
}

namespace {

template <typename T>
int dalloc(T **p, size_t count)
{
    *p = (T *)ba_dmalloc(sizeof(T) * (count ? count : 1));
    return *p ? 0 : -(int)hipErrorOutOfMemory;
}

template <typename T>
int upload(T *dst, const T *src, size_t count, hipStream_t s)
{
    if (count == 0) return 0;
    hipError_t e = hipMemcpyAsync(dst, src, sizeof(T) * count, hipMemcpyHostToDevice, s);
    return e == hipSuccess ? 0 : -(int)e;
}

template <typename T>
int download(T *dst, const T *src, size_t count, hipStream_t s)
{
    if (count == 0) return 0;
    hipError_t e = hipMemcpyAsync(dst, src, sizeof(T) * count, hipMemcpyDeviceToHost, s);
    return e == hipSuccess ? 0 : -(int)e;
}

#define TRY(x)                                                                      \
    do {                                                                            \
        int rc__ = (x);                                                             \
        if (rc__) return rc__;                                                      \
    } while (0)

// Observation list sorted point-major: points ascending, cameras ascending
// within a point (the order of the reference's column-major n x m loops).
struct host_obs {
    std::vector<int> pt, cam;
    std::vector<double> x;
};

int sort_obs(const vlgba_problem *p, host_obs &h)
{
    const long long N = p->num_obs;
    // already point-major with cameras ascending within a point (the growing
    // replay's subsets, bundle_euclid's visibility order): a copy
    bool sorted = true;
    for (long long o = 0; o < N && sorted; o++) {
        const int i = p->obs_pt[o], j = p->obs_cam[o];
        if (i < 0 || i >= p->n || j < 0 || j >= p->m) return VLGBA_E_ARG;
        if (o > 0) {
            const int i0 = p->obs_pt[o - 1], j0 = p->obs_cam[o - 1];
            if (i < i0 || (i == i0 && j < j0)) sorted = false;
            else if (i == i0 && j == j0) return VLGBA_E_ORDER;
        }
    }
    if (sorted) {
        h.pt.assign(p->obs_pt, p->obs_pt + N);
        h.cam.assign(p->obs_cam, p->obs_cam + N);
        h.x.assign(p->obs_x, p->obs_x + 2 * N);
        return 0;
    }
    std::vector<long long> cnt(p->n + 1, 0);
    for (long long o = 0; o < N; o++) {
        const int i = p->obs_pt[o], j = p->obs_cam[o];
        if (i < 0 || i >= p->n || j < 0 || j >= p->m) return VLGBA_E_ARG;
        cnt[i + 1]++;
    }
    for (int i = 0; i < p->n; i++) cnt[i + 1] += cnt[i];
    std::vector<long long> pos(cnt.begin(), cnt.end() - 1);
    std::vector<long long> perm(N);
    for (long long o = 0; o < N; o++) perm[pos[p->obs_pt[o]]++] = o;
    h.pt.resize(N);
    h.cam.resize(N);
    h.x.resize(2 * N);
    for (int i = 0; i < p->n; i++) {
        std::sort(perm.begin() + cnt[i], perm.begin() + cnt[i + 1],
                  [&](long long u, long long v) { return p->obs_cam[u] < p->obs_cam[v]; });
        for (long long q = cnt[i]; q < cnt[i + 1]; q++) {
            const long long o = perm[q];
            if (q > cnt[i] && p->obs_cam[o] == h.cam[q - 1]) return VLGBA_E_ORDER;
            h.pt[q] = i;
            h.cam[q] = p->obs_cam[o];
            h.x[2 * q] = p->obs_x[2 * o];
            h.x[2 * q + 1] = p->obs_x[2 * o + 1];
        }
    }
    return 0;
}

// Co-visible camera-pair blocks and their term lists (obs pairs, point
// ascending).  lower: blocks j >= k only (the Cholesky reads the lower
// triangle); otherwise all ordered pairs (stage-2 entry: full S like
// mex_bundle_2_Se_.c).  The block SET comes from all observations (so every
// rank agrees on the packed layout); terms only from observations [o0, o1).
struct host_blocks {
    std::vector<int> jk, ptr, term;
    int m = 0;
    bool dense_tab = true;
    std::vector<int> tab;                                // m*m block ids (dense)
    std::vector<std::vector<std::pair<int, int>>> rows;  // sparse fallback: (k, id)
    // empty, keeping the vectors' capacity (a context per growing-replay solve:
    // reused storage is not page-faulted in again, ctx_setup's per-thread pool)
    // The dense table stays allocated and all -1 between contexts: reset()
    // clears the entries this context's blocks set (O(blocks) instead of
    // rewriting m x m ints -- 3.2 MB at 900 cameras -- per context).
    void reset()
    {
        if (dense_tab && !tab.empty())
            for (size_t q = 0; q + 1 < jk.size(); q += 2) tab[(size_t)jk[q] * m + jk[q + 1]] = -1;
        jk.clear();
        ptr.clear();
        term.clear();
        m = 0;
        dense_tab = true;
        rows.clear();
    }
    int find(int j, int k) const
    {
        if (dense_tab) return tab[(size_t)j * m + k];
        for (auto &pr : rows[j])
            if (pr.first == k) return pr.second;
        return -1;
    }
    int insert(int j, int k)
    {
        int id = find(j, k);
        if (id >= 0) return id;
        id = (int)jk.size() / 2;
        jk.push_back(j);
        jk.push_back(k);
        if (dense_tab) tab[(size_t)j * m + k] = id;
        else rows[j].push_back({k, id});
        return id;
    }
};

void build_blocks(int m, const std::vector<int> &pt_ptr_all, const std::vector<int> &cam_all,
                  int p0, int p1, long long obs_base, bool lower, bool all_diag, bool need_terms,
                  host_blocks &hb)
{
    const int n = (int)pt_ptr_all.size() - 1;
    hb.m = m;
    hb.dense_tab = (long long)m * m <= (1LL << 26);
    if (hb.dense_tab && hb.tab.size() < (size_t)m * m)   // (else all -1 already: reset)
        hb.tab.assign((size_t)m * m, -1);
    else hb.rows.resize(m);
    auto find = [&](int j, int k) -> int { return hb.find(j, k); };
    // canonical block ids, (k, j) ascending: independent of the point order,
    // so ranks that order their own points differently (order_points_by_kind)
    // agree on the packed layout of the all-reduced blocks
    if (lower && hb.dense_tab) {
        // the lower block set as one bit row per column k (bit j: block (j, k),
        // j >= k), each point's cameras OR-ed in as a word mask over the span
        // of its track (cameras ascending within a point): O(track x span / 64)
        // per point instead of one table insert per camera pair, then the ids
        // handed out row by row = (k, j) ascending
        const int nw = (m + 63) / 64;
        std::vector<unsigned long long> rowb((size_t)m * nw, 0ull), mask(nw, 0ull);
        if (all_diag)
            for (int j = 0; j < m; j++) rowb[(size_t)j * nw + (j >> 6)] |= 1ull << (j & 63);
        for (int i = 0; i < n; i++) {
            const int a0 = pt_ptr_all[i], a1 = pt_ptr_all[i + 1];
            if (a1 <= a0) continue;
            const int w0 = cam_all[a0] >> 6, w1 = cam_all[a1 - 1] >> 6;
            for (int a = a0; a < a1; a++) mask[cam_all[a] >> 6] |= 1ull << (cam_all[a] & 63);
            for (int a = a0; a < a1; a++) {
                unsigned long long *row = &rowb[(size_t)cam_all[a] * nw];
                for (int w = w0; w <= w1; w++) row[w] |= mask[w];
            }
            for (int w = w0; w <= w1; w++) mask[w] = 0ull;
        }
        for (int k = 0; k < m; k++) {
            const unsigned long long *row = &rowb[(size_t)k * nw];
            for (int w = k >> 6; w < nw; w++) {
                unsigned long long bits = row[w];
                if (w == (k >> 6)) bits &= ~0ull << (k & 63);   // j >= k only
                while (bits) {
                    const int j = 64 * w + __builtin_ctzll(bits);
                    bits &= bits - 1;
                    hb.tab[(size_t)j * m + k] = (int)hb.jk.size() / 2;
                    hb.jk.push_back(j);
                    hb.jk.push_back(k);
                }
            }
        }
    } else {
        if (all_diag)
            for (int j = 0; j < m; j++) hb.insert(j, j);
        for (int i = 0; i < n; i++)
            for (int a = pt_ptr_all[i]; a < pt_ptr_all[i + 1]; a++)
                for (int b = pt_ptr_all[i]; b < pt_ptr_all[i + 1]; b++) {
                    const int j = cam_all[a], k = cam_all[b];
                    if (lower && j < k) continue;
                    hb.insert(j, k);
                }
        const int nb0 = (int)hb.jk.size() / 2;
        std::vector<int> ord(nb0);
        std::iota(ord.begin(), ord.end(), 0);
        std::sort(ord.begin(), ord.end(), [&](int u, int v) {
            const int ku = hb.jk[2 * u + 1], kv = hb.jk[2 * v + 1];
            return ku != kv ? ku < kv : hb.jk[2 * u] < hb.jk[2 * v];
        });
        std::vector<int> jk2(2 * (size_t)nb0);
        for (int q = 0; q < nb0; q++) {
            jk2[2 * q] = hb.jk[2 * ord[q]];
            jk2[2 * q + 1] = hb.jk[2 * ord[q] + 1];
        }
        hb.jk.swap(jk2);
        if (hb.dense_tab) {
            for (int q = 0; q < nb0; q++) hb.tab[(size_t)hb.jk[2 * q] * m + hb.jk[2 * q + 1]] = q;
        } else {
            for (auto &r : hb.rows) r.clear();
            for (int q = 0; q < nb0; q++) hb.rows[hb.jk[2 * q]].push_back({hb.jk[2 * q + 1], q});
        }
    }
    const int nb = (int)hb.jk.size() / 2;
    if (!need_terms) {
        hb.ptr.assign(nb + 1, 0);
        return;
    }
    std::vector<long long> cnt(nb + 1, 0);
    for (int i = p0; i < p1; i++)
        for (int a = pt_ptr_all[i]; a < pt_ptr_all[i + 1]; a++)
            for (int b = pt_ptr_all[i]; b < pt_ptr_all[i + 1]; b++) {
                const int j = cam_all[a], k = cam_all[b];
                if (lower && j < k) continue;
                cnt[find(j, k) + 1]++;
            }
    for (int q = 0; q < nb; q++) cnt[q + 1] += cnt[q];
    hb.ptr.resize(nb + 1);
    for (int q = 0; q <= nb; q++) hb.ptr[q] = (int)cnt[q];
    hb.term.resize(2 * (size_t)cnt[nb]);
    std::vector<long long> pos(cnt.begin(), cnt.end() - 1);
    for (int i = p0; i < p1; i++)   // points ascending => terms ascending per block
        for (int a = pt_ptr_all[i]; a < pt_ptr_all[i + 1]; a++)
            for (int b = pt_ptr_all[i]; b < pt_ptr_all[i + 1]; b++) {
                const int j = cam_all[a], k = cam_all[b];
                if (lower && j < k) continue;
                const long long s = pos[find(j, k)]++;
                hb.term[2 * s] = (int)(a - obs_base);
                hb.term[2 * s + 1] = (int)(b - obs_base);
            }
}

// Chunk plan of the fast Schur path for the local points (pt_ptr local,
// cam local observation cameras).  Points [0, p_split) form MFMA chunks
// (k_schur_mfma), points [p_split, n) per-term chunks (k_schur_group); the
// chunk and group sequences keep that order, so the MFMA groups are
// [0, ngrp_mf) and the term groups [ngrp_mf, ngrp).  Returns false when a
// point does not fit its chunk kind (the caller then uses the ordered kernels).
struct host_plan {
    std::vector<int> ch_pt, ch_slot, ch_eslot, slot_blk, slot_tptr, eslot_optr;
    std::vector<unsigned short> slot_term, eslot_obs;
    std::vector<int> cam_eptr, cam_eslots;
    int max_terms = 0, max_slots = 0;   // per chunk (LDS staging size)
    long long n_terms = 0;              // (obs, obs) Schur terms of all chunks
    // Schur groups: consecutive chunks whose co-visible blocks ("group slots")
    // and cameras ("group e-slots") are accumulated in LDS across the group
    std::vector<int> grp_ch, grp_gs, grp_ge;      // [ngrp+1] ranges
    std::vector<unsigned short> cs_g, ce_g;        // chunk slot / e-slot -> group-local id
    std::vector<int> gslot_blk, gecam;             // [ngs], [nge]
    std::vector<int> blk_gptr, blk_gslots, cam_gptr, cam_gslots;
    int grp_max_s = 0, grp_max_e = 0;             // largest accumulated term group
    int mf_max_s = 0, mf_max_e = 0;               // largest MFMA group
    int nch_mf = 0, ngrp_mf = 0;                  // leading MFMA chunks / groups
    // long tracks (points [p_long, n)): each split into segment chunks of <=
    // BA_CH_OBS observations (after the regular chunks: chunk ids
    // [nch_reg, nch_reg + nseg)); their Schur terms are group slots of their
    // own, one per (obs, obs) pair, and one group e-slot per observation
    int nch_reg = 0, nseg = 0;
    std::vector<int> seg_pt, seg_long;            // [nseg] point / long index
    std::vector<int> long_pt, long_o0, long_seg0; // [nl], [nl+1], [nl+1]
    std::vector<int> long_ebase;                  // [nl] first group e-slot
    std::vector<int> cam_lptr, cam_lobs, cam_ltrk; // per camera its long observations
    int max_lcam = 0;                             // (long-obs index, track), track order
    // per chunk one contiguous metadata record (one coalesced prefetch):
    //   [np | nobs << 16][ns | nes << 16][nterm][neobs] soff[ns+1] eoff[nes+1]
    //   sgl[ns] egl[nes] lpt[nobs] term[nterm] (y | w << 16) eobl[neobs]
    std::vector<unsigned> blob;
    std::vector<int> ch_blob, ch_obase;            // [nch+1]
    int max_blob = 0;      // term chunks: largest record
    int mf_max_blob = 0;   // MFMA groups: largest group record block (staged in LDS)
    // empty, keeping every vector's capacity (host_blocks::reset)
    void reset()
    {
        for (std::vector<int> *v :
             {&ch_pt, &ch_slot, &ch_eslot, &slot_blk, &slot_tptr, &eslot_optr,
              &cam_eptr, &cam_eslots, &grp_ch, &grp_gs, &grp_ge, &gslot_blk, &gecam,
              &blk_gptr, &blk_gslots, &cam_gptr, &cam_gslots, &seg_pt, &seg_long, &long_pt,
              &long_o0, &long_seg0, &long_ebase, &cam_lptr, &cam_lobs, &cam_ltrk, &ch_blob,
              &ch_obase})
            v->clear();
        for (std::vector<unsigned short> *v : {&slot_term, &eslot_obs, &cs_g, &ce_g}) v->clear();
        blob.clear();
        max_terms = max_slots = 0;
        n_terms = 0;
        grp_max_s = grp_max_e = mf_max_s = mf_max_e = nch_mf = ngrp_mf = 0;
        nch_reg = nseg = max_lcam = max_blob = mf_max_blob = 0;
    }
};

static int plan_threads(long long work, long long min_work);
template <typename F>
static void parallel_ranges(int n, int nthr, F f, const std::vector<long long> *wpre);

// counting sort of ids by key: ptr[nkey+1], list of ids in ascending id order
// per key (large inputs: per-thread counts over contiguous id ranges, each
// thread's ids placed after those of the ranges before it: the same order)
static void bucket(const std::vector<int> &key, int nkey, std::vector<int> &ptr,
                   std::vector<int> &list)
{
    const int n = (int)key.size();
    const int T = std::min(plan_threads(n, 200000), std::max(1, (int)(4LL * n / (nkey + 1))));
    ptr.assign(nkey + 1, 0);
    list.resize(key.size());
    if (T <= 1) {
        for (int k : key) ptr[k + 1]++;
        for (int q = 0; q < nkey; q++) ptr[q + 1] += ptr[q];
        std::vector<int> pos(ptr.begin(), ptr.end() - 1);
        for (int s = 0; s < n; s++) list[pos[key[s]]++] = s;
        return;
    }
    std::vector<std::vector<int>> cnt(T);
    parallel_ranges(n, T, [&](int t, int s0, int s1) {
        cnt[t].assign(nkey, 0);
        for (int s = s0; s < s1; s++) cnt[t][key[s]]++;
    }, nullptr);
    for (int k = 0; k < nkey; k++) {   // cnt[t][k] <- start of thread t's ids of key k
        int at = ptr[k];
        for (int t = 0; t < T; t++) {
            const int c = cnt[t][k];
            cnt[t][k] = at;
            at += c;
        }
        ptr[k + 1] = at;
    }
    parallel_ranges(n, T, [&](int t, int s0, int s1) {
        std::vector<int> &pos = cnt[t];
        for (int s = s0; s < s1; s++) list[pos[key[s]]++] = s;
    }, nullptr);
}

// phase times of build_plan on stderr (tools/bench_plan.sh builds with it)
#ifdef BA_PLAN_TIMING
#define PLAN_T0 auto plan_t0_ = std::chrono::steady_clock::now()
#define PLAN_T(w)                                                                           \
    do {                                                                                    \
        const auto t_ = std::chrono::steady_clock::now();                                   \
        std::fprintf(stderr, "   %-14s %7.2f ms\n", w,                                     \
                     std::chrono::duration<double, std::milli>(t_ - plan_t0_).count());     \
        plan_t0_ = t_;                                                                      \
    } while (0)
#else
#define PLAN_T0
#define PLAN_T(w)
#endif

// Host threads of a context's plan: VLGBA_HOST_THREADS, else OMP_NUM_THREADS
// (the GPU box's CPU share), else the hardware's, at most 16; fewer when the
// work has fewer than min_work items per thread.
static int plan_threads(long long work, long long min_work)
{
    static const int cap = [] {
        int v = 0;
        if (const char *e = std::getenv("VLGBA_HOST_THREADS")) v = std::atoi(e);
        if (v <= 0)
            if (const char *e = std::getenv("OMP_NUM_THREADS")) v = std::atoi(e);
        if (v <= 0) v = (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(v, 16));
    }();
    return (int)std::max(1LL, std::min<long long>(cap, work / std::max(1LL, min_work)));
}

// The host planner's worker threads: created once and kept (a context is
// created per growing-replay solve, and spawning 15 threads per plan phase
// cost more than some phases).  Two pools, one job each at a time: the
// replay builds two contexts side by side (its two prefetch workers); a
// caller that finds both busy (more concurrent creations, e.g. rank
// threads), or a forked child (the pools' threads stayed in the parent), runs
// its job on threads of its own instead.
class plan_pool {
  public:
    // f(t) for t in [0, nthr): t = 0 on the calling thread; false (nothing
    // run) if this pool is busy or unusable here
    bool try_run(int nthr, const std::function<void(int)> &f)
    {
        std::unique_lock<std::mutex> busy(job_mu_, std::defer_lock);
        if (getpid() != pid_ || nthr - 1 > kMax || !busy.try_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)th_.size() < nthr - 1) {
                const int id = (int)th_.size() + 1;
                th_.emplace_back([this, id] { loop(id); });
            }
            job_ = &f;
            njob_ = nthr;
            pending_ = nthr - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
        return true;
    }

  private:
    static constexpr int kMax = 15;
    void loop(int id)
    {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)> *f = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (id < njob_) f = job_;
            }
            if (!f) continue;
            (*f)(id);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    const pid_t pid_ = getpid();
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(int)> *job_ = nullptr;
    int njob_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
};

static void plan_run(int nthr, const std::function<void(int)> &f)
{
    static plan_pool *pools = new plan_pool[2];   // never destroyed: no join at exit
    for (int q = 0; q < 2; q++)
        if (pools[q].try_run(nthr, f)) return;
    std::vector<std::thread> th;   // threads of our own
    for (int t = 1; t < nthr; t++) th.emplace_back(f, t);
    f(0);
    for (auto &x : th) x.join();
}

// f(t, lo, hi) on nthr contiguous ranges of [0, n) (thread t takes range t;
// the calling thread takes range 0), of equal work when wpre (the prefix sums
// of per-item work, n + 1 entries) is given, else of equal length
template <typename F>
static void parallel_ranges(int n, int nthr, F f, const std::vector<long long> *wpre)
{
    if (nthr <= 1) {
        f(0, 0, n);
        return;
    }
    std::vector<int> cut(nthr + 1, n);
    cut[0] = 0;
    for (int t = 1; t < nthr; t++) {
        if (wpre) {
            const long long target = (*wpre)[n] * t / nthr;
            cut[t] = (int)(std::lower_bound(wpre->begin(), wpre->begin() + n + 1, target) -
                           wpre->begin());
        } else {
            cut[t] = (int)((long long)n * t / nthr);
        }
        cut[t] = std::max(cut[t], cut[t - 1]);
    }
    plan_run(nthr, [&](int t) { f(t, cut[t], cut[t + 1]); });
}

// MFMA chunks (points below p_split): at most BA_MF_PTS points and cmax
// cameras per chunk (the chunk's dense Y / W fit one K = 64 slab of
// 16 * BA_MF_RT(na) rows); their metadata records are the dense-layout ones
// described at build of P.blob below.
bool build_plan(int m, int na, const std::vector<int> &lptr, const std::vector<int> &lcam,
                const host_blocks &hb, host_plan &P, int cmax, int p_split, int p_long)
{
    const int n_all = (int)lptr.size() - 1;
    const int n = p_long;   // regular chunks cover points [0, p_long)
    const int nb = (int)hb.jk.size() / 2;
    if (cmax <= 0) p_split = 0;
    auto pt_terms = [&](int i) {
        const long long k = lptr[i + 1] - lptr[i];
        return k * (k + 1) / 2;
    };
    for (int i = 0; i < n; i++)
        if (lptr[i + 1] - lptr[i] > BA_CH_OBS || pt_terms(i) > BA_CH_TERMS ||
            (i < p_split && lptr[i + 1] - lptr[i] > cmax))
            return false;
    PLAN_T0;
    // chunk boundaries (sequential: the MFMA chunking follows the camera sets)
    std::vector<int> cbeg, cend;
    std::vector<char> cmf;
    {
        std::vector<int> cam_stamp(m, -1);   // chunk camera set (MFMA chunking)
        P.max_terms = 0;
        int p = 0;
        while (p < n) {
            const bool mf = p < p_split;                // chunk kind
            const int pend = mf ? p_split : n;
            const int pts_max = mf ? BA_MF_PTS : BA_CH_PTS;
            const int obase = lptr[p];
            int q = p;
            long long nterm = 0;
            int ncam = 0;
            bool uniform = true;   // every point so far sees exactly the first point's cameras
            auto same_cams = [&](int i1, int i2) {
                if (lptr[i1 + 1] - lptr[i1] != lptr[i2 + 1] - lptr[i2]) return false;
                for (int a = 0; a < lptr[i1 + 1] - lptr[i1]; a++)
                    if (lcam[lptr[i1] + a] != lcam[lptr[i2] + a]) return false;
                return true;
            };
            while (q < pend && q - p < pts_max && lptr[q + 1] - obase <= BA_CH_OBS &&
                   nterm + pt_terms(q) <= BA_CH_TERMS) {
                if (mf) {
                    // a run of points with one camera list (video-like tracks) keeps
                    // its chunks to itself: its MFMA sums stay in registers across
                    // chunks
                    const bool same = q == p || same_cams(p, q);
                    if (uniform && !same && q - p >= 4) break;
                    uniform = uniform && same;
                    int add = 0;
                    for (int a = lptr[q]; a < lptr[q + 1]; a++) add += cam_stamp[lcam[a]] != p;
                    if (ncam + add > cmax) break;
                    for (int a = lptr[q]; a < lptr[q + 1]; a++) cam_stamp[lcam[a]] = p;
                    ncam += add;
                }
                nterm += pt_terms(q++);
            }
            P.max_terms = std::max(P.max_terms, (int)nterm);
            P.n_terms += nterm;
            cbeg.push_back(p);
            cend.push_back(q);
            cmf.push_back(mf ? 1 : 0);
            p = q;
        }
    }
    PLAN_T("boundaries");
    // per chunk, in parallel over ranges of chunks (each thread's output is
    // contiguous in chunk order, so the ranges concatenate to the sequential
    // plan): pass 1 the chunk's slots (co-visible blocks, by first touch) and
    // e-slots (cameras) with their term / observation counts; pass 2 the
    // per-term lists (term chunks only: the MFMA records are dense) and the
    // per-camera observation lists, grouped by slot / e-slot in that order
    const int nchk = (int)cbeg.size();
    // (cache-line aligned: every push_back writes a vector header, and the
    // headers of neighbouring threads' outputs must not share a line)
    struct alignas(128) chunk_out {
        std::vector<int> blk, tcnt, cam, ecnt, ns, nes;
        std::vector<unsigned short> term, eobs;
        void clear()
        {
            for (std::vector<int> *v : {&blk, &tcnt, &cam, &ecnt, &ns, &nes}) v->clear();
            term.clear();
            eobs.clear();
        }
    };
    std::vector<long long> cwork(nchk + 1, 0);   // per chunk: its terms and observations
    for (int c = 0; c < nchk; c++) {
        long long w = lptr[cend[c]] - lptr[cbeg[c]];
        for (int i = cbeg[c]; i < cend[c]; i++) w += pt_terms(i);
        cwork[c + 1] = cwork[c] + w;
    }
    const int nthr = plan_threads(cwork[nchk], 20000);
    // the per-thread outputs live in the calling thread's scratch (capacity kept
    // from one context to the next: no page faults on the replay's plans)
    // (a reference: the pool threads' lambda must reach THIS thread's scratch,
    // not their own thread_local instance)
    static thread_local std::vector<chunk_out> co_tl;
    std::vector<chunk_out> &co = co_tl;
    if ((int)co.size() < nthr) co.resize(nthr);
    for (chunk_out &o : co) o.clear();
#ifdef BA_PLAN_TIMING
    std::vector<double> thr_ms(nthr, 0.0), thr_start(nthr, 0.0);
    PLAN_T("chunks prep");
    const auto tpr0 = std::chrono::steady_clock::now();
#endif
    parallel_ranges(nchk, nthr, [&](int t, int c0, int c1) {
#ifdef BA_PLAN_TIMING
        const auto tt0 = std::chrono::steady_clock::now();
        thr_start[t] = std::chrono::duration<double, std::milli>(tt0 - tpr0).count();
        struct tdone {
            std::chrono::steady_clock::time_point t0;
            double *out;
            ~tdone()
            {
                *out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                                 t0).count();
            }
        } tdone_{tt0, &thr_ms[t]};
#endif
        chunk_out &o = co[t];
        // per chunk: its cameras' local ids (e-slots, by first touch) and a
        // local nes x nes table of slot ids -- one global block lookup per
        // camera pair of the chunk instead of two per (obs, obs) term (the
        // m x m table does not stay in cache at ~1000 cameras); slots are
        // still numbered by first touch in (point, a, b) order
        std::vector<int> eslot_of(m, -1), tpos, epos, le, lslot;
        for (int c = c0; c < c1; c++) {
            const int p = cbeg[c], q = cend[c], obase = lptr[p], nob = lptr[q] - obase;
            const bool mf = cmf[c] != 0;
            const size_t s0 = o.blk.size(), e0 = o.cam.size();
            le.resize(nob);
            for (int a = obase; a < obase + nob; a++) {
                const int j = lcam[a];
                if (eslot_of[j] < 0) {
                    eslot_of[j] = (int)(o.cam.size() - e0);
                    o.cam.push_back(j);
                    o.ecnt.push_back(0);
                }
                o.ecnt[e0 + eslot_of[j]]++;
                le[a - obase] = eslot_of[j];
            }
            const int nce = (int)(o.cam.size() - e0);
            lslot.assign((size_t)nce * nce, -1);
            for (int i = p; i < q; i++)
                for (int a = lptr[i]; a < lptr[i + 1]; a++) {
                    const int j = lcam[a], ea = le[a - obase];
                    for (int b = lptr[i]; b < lptr[i + 1]; b++) {
                        const int k = lcam[b];
                        if (j < k) continue;
                        int &sl = lslot[(size_t)ea * nce + le[b - obase]];
                        if (sl < 0) {
                            sl = (int)(o.blk.size() - s0);
                            o.blk.push_back(hb.find(j, k));
                            o.tcnt.push_back(0);
                        }
                        o.tcnt[s0 + sl]++;
                    }
                }
            const int ns = (int)(o.blk.size() - s0), nes = (int)(o.cam.size() - e0);
            o.ns.push_back(ns);
            o.nes.push_back(nes);
            tpos.assign(ns + 1, 0);
            epos.assign(nes + 1, 0);
            for (int sl = 0; sl < ns; sl++) {
                if (mf) o.tcnt[s0 + sl] = 0;   // the MFMA records are dense: no term lists
                tpos[sl + 1] = tpos[sl] + o.tcnt[s0 + sl];
            }
            for (int e = 0; e < nes; e++) epos[e + 1] = epos[e] + o.ecnt[e0 + e];
            const size_t tb = o.term.size() / 2, ub = o.eobs.size();
            o.term.resize(2 * (tb + tpos[ns]));
            o.eobs.resize(ub + epos[nes]);
            for (int i = p; i < q; i++)
                for (int a = lptr[i]; a < lptr[i + 1]; a++) {
                    const int j = lcam[a], ea = le[a - obase];
                    o.eobs[ub + epos[ea]++] = (unsigned short)(a - obase);
                    if (mf) continue;
                    for (int b = lptr[i]; b < lptr[i + 1]; b++) {
                        if (j < lcam[b]) continue;
                        const size_t at = tb + tpos[lslot[(size_t)ea * nce + le[b - obase]]]++;
                        o.term[2 * at] = (unsigned short)(a - obase);
                        o.term[2 * at + 1] = (unsigned short)(b - obase);
                    }
                }
            for (size_t e = e0; e < o.cam.size(); e++) eslot_of[o.cam[e]] = -1;
        }
    }, &cwork);
#ifdef BA_PLAN_TIMING
    std::fprintf(stderr, "   (chunk threads:");
    for (int q = 0; q < nthr; q++) std::fprintf(stderr, " %.2f+%.2f", thr_start[q], thr_ms[q]);
    std::fprintf(stderr, " ms)\n");
#endif
    PLAN_T("chunks");
    // concatenate in chunk order: every thread's output block has a known
    // offset (sizes summed in thread order), so the blocks are copied -- and
    // their slot / e-slot prefix sums and chunk ranges formed -- in parallel
    // (element by element push_backs cost ~2 ms at cfg5x-900, sequentially)
    {
        const int NO = (int)co.size();
        std::vector<size_t> ob(NO + 1, 0), oc(NO + 1, 0), ot(NO + 1, 0), ou(NO + 1, 0),
            och(NO + 1, 0);
        for (int t = 0; t < NO; t++) {
            ob[t + 1] = ob[t] + co[t].blk.size();
            oc[t + 1] = oc[t] + co[t].cam.size();
            ot[t + 1] = ot[t] + co[t].term.size();
            ou[t + 1] = ou[t] + co[t].eobs.size();
            och[t + 1] = och[t] + co[t].ns.size();
        }
        P.slot_blk.resize(ob[NO]);
        P.slot_tptr.resize(ob[NO] + 1);
        P.cam_eslots.resize(oc[NO]);
        P.eslot_optr.resize(oc[NO] + 1);
        P.slot_term.resize(ot[NO]);
        P.eslot_obs.resize(ou[NO]);
        P.ch_pt.resize(och[NO] + 1);
        P.ch_slot.resize(och[NO] + 1);
        P.ch_eslot.resize(och[NO] + 1);
        P.slot_tptr[0] = P.eslot_optr[0] = 0;
        P.ch_pt[0] = P.ch_slot[0] = P.ch_eslot[0] = 0;
        std::vector<int> tmax(NO, 0);
        auto copy_block = [&](int t) {
            const chunk_out &o = co[t];
            std::copy(o.blk.begin(), o.blk.end(), P.slot_blk.begin() + ob[t]);
            int acc = (int)(ot[t] / 2);   // term pairs before this block
            for (size_t q = 0; q < o.tcnt.size(); q++) P.slot_tptr[ob[t] + 1 + q] = acc += o.tcnt[q];
            std::copy(o.cam.begin(), o.cam.end(), P.cam_eslots.begin() + oc[t]);
            acc = (int)ou[t];
            for (size_t q = 0; q < o.ecnt.size(); q++) P.eslot_optr[oc[t] + 1 + q] = acc += o.ecnt[q];
            std::copy(o.term.begin(), o.term.end(), P.slot_term.begin() + ot[t]);
            std::copy(o.eobs.begin(), o.eobs.end(), P.eslot_obs.begin() + ou[t]);
            int sa = (int)ob[t], ea = (int)oc[t];
            for (size_t u = 0; u < o.ns.size(); u++) {
                const size_t c = och[t] + u;
                tmax[t] = std::max(tmax[t], o.ns[u]);
                P.ch_pt[c + 1] = cend[c];
                P.ch_slot[c + 1] = sa += o.ns[u];
                P.ch_eslot[c + 1] = ea += o.nes[u];
            }
        };
        const int nct = std::min(NO, plan_threads((long long)(ob[NO] + ot[NO] + ou[NO]), 50000));
        plan_run(nct, [&](int w) {
            for (int t = w; t < NO; t += nct) copy_block(t);
        });
        P.max_slots = 0;
        for (int t = 0; t < NO; t++) P.max_slots = std::max(P.max_slots, tmax[t]);
        for (int c = 0; c < nchk; c++)
            if (cmf[c]) P.nch_mf++;
    }
    PLAN_T("concat");
    // long tracks: segment chunks (one point each, <= BA_CH_OBS observations;
    // every observation its own camera slot: a point sees a camera once)
    P.nch_reg = (int)P.ch_pt.size() - 1;
    P.long_o0.assign(1, lptr[p_long]);
    P.long_seg0.assign(1, 0);
    for (int i = p_long; i < n_all; i++) {
        const int l = (int)P.long_pt.size();
        P.long_pt.push_back(i);
        for (int o = lptr[i]; o < lptr[i + 1]; o += BA_CH_OBS) {
            const int o1 = std::min(o + BA_CH_OBS, lptr[i + 1]);
            for (int a = o; a < o1; a++) {
                P.eslot_obs.push_back((unsigned short)(a - o));
                P.eslot_optr.push_back((int)P.eslot_obs.size());
                P.cam_eslots.push_back(lcam[a]);
            }
            P.ch_eslot.push_back((int)P.eslot_optr.size() - 1);
            P.seg_pt.push_back(i);
            P.seg_long.push_back(l);
            P.nseg++;
        }
        P.long_o0.push_back(lptr[i + 1]);
        P.long_seg0.push_back(P.nseg);
    }
    // per camera: its e-slots in chunk order (cam_eslots currently = camera of
    // e-slot) -- a counting sort that keeps the id order (bucket: threads over
    // id ranges for large inputs).  (The per-block lists of the chunk slots are
    // not built: the block sums read the group slots, blk_gptr / blk_gslots.)
    std::vector<int> ecam;
    ecam.swap(P.cam_eslots);
    bucket(ecam, m, P.cam_eptr, P.cam_eslots);
    const int ns = (int)P.slot_blk.size(), nes = (int)P.eslot_optr.size() - 1;
    PLAN_T("blk lists");
    // Schur groups (greedy): at most gs_cap distinct blocks (LDS accumulators),
    // BA_GE_CAP cameras and gmax chunks (>= ~2048 groups keep the chip busy).
    // A chunk with more than gs_cap blocks forms a group of its own whose
    // partials go straight to HBM ("direct" group).
    const int nch = (int)P.ch_pt.size() - 1;
    std::vector<int> gslot_of(nb, -1), gcam_of(m, -1);
    P.cs_g.assign(ns, 0);
    P.ce_g.assign(nes, 0);
    P.grp_ch.assign(1, 0);
    P.grp_gs.assign(1, 0);
    P.grp_ge.assign(1, 0);
    // The MFMA segment's chunks are spread evenly over BA_MF_GROUPS groups
    // (fractional: group k ends near chunk (k + 1) nseg / G): one workgroup
    // per slot of k_schur_mfma's 3 x 256 CUs, no partly filled last round
    // (config 3: 1953 groups of 13 chunks -- 2.54 rounds -- took 179-183 us,
    // 1536 groups 167-169, 768 groups 155; 1024 / 2304 / 3072: 182-187,
    // profiles/r05i_*, r05j_*).  The term segment keeps BA_GROUPS' cap.
    // VLGBA_SCHUR_GROUPS overrides G (measurement).
    static const int Genv = [] {
        const char *e = std::getenv("VLGBA_SCHUR_GROUPS");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? v : 0;
    }();
    int seg0 = 0, kseg = 0;
    for (int c = 0; c < nch;) {
        const bool mf = c < P.nch_mf;
        const int cend = mf ? P.nch_mf : nch, nseg = mf ? P.nch_mf : nch - P.nch_mf;
        if (c == 0 || c == P.nch_mf) seg0 = c, kseg = 0;
        // the MFMA kernel has no direct mode: one chunk's blocks must always fit
        const int gs_cap = mf ? std::max(BA_MF_GACC / (na * na), cmax * (cmax + 1) / 2)
                              : BA_GACC / (na * na);
        const int G = Genv ? Genv : (mf ? BA_MF_GROUPS : 0);
        const long long tend = G ? seg0 + ((long long)(kseg + 1) * nseg + G - 1) / G : 0;
        const int gmax = G ? (int)std::min<long long>(BA_GROUP_CH, std::max<long long>(1, tend - c))
                           : std::min(BA_GROUP_CH, std::max(1, (nseg + BA_GROUPS - 1) / BA_GROUPS));
        kseg++;
        const int ge_cap = mf ? std::max(BA_MF_GE_CAP, cmax) : BA_GE_CAP;
        if (gmax == 1) {
            // one chunk per group: its slots and e-slots are distinct blocks /
            // cameras already, so the group's lists are the chunk's (what the
            // general loop below builds, without its table lookups)
            const int s0 = P.ch_slot[c], s1 = P.ch_slot[c + 1];
            const int e0 = P.ch_eslot[c], e1 = P.ch_eslot[c + 1];
            P.gslot_blk.insert(P.gslot_blk.end(), P.slot_blk.begin() + s0,
                               P.slot_blk.begin() + s1);
            for (int q = s0; q < s1; q++) P.cs_g[q] = (unsigned short)(q - s0);
            P.gecam.insert(P.gecam.end(), ecam.begin() + e0, ecam.begin() + e1);
            for (int q = e0; q < e1; q++) P.ce_g[q] = (unsigned short)(q - e0);
            const int ngs_ = s1 - s0, nge_ = e1 - e0;
            if (mf) {
                P.mf_max_s = std::max(P.mf_max_s, ngs_);
                P.mf_max_e = std::max(P.mf_max_e, nge_);
                P.ngrp_mf++;
            } else if (ngs_ <= gs_cap) {
                P.grp_max_s = std::max(P.grp_max_s, ngs_);
                P.grp_max_e = std::max(P.grp_max_e, nge_);
            }
            P.grp_ch.push_back(c + 1);
            P.grp_gs.push_back((int)P.gslot_blk.size());
            P.grp_ge.push_back((int)P.gecam.size());
            c++;
            continue;
        }
        std::vector<int> gs, ge;
        int d = c;
        for (; d < cend && d - c < gmax; d++) {
            int new_s = 0, new_e = 0;
            for (int s = P.ch_slot[d]; s < P.ch_slot[d + 1]; s++) new_s += gslot_of[P.slot_blk[s]] < 0;
            for (int e = P.ch_eslot[d]; e < P.ch_eslot[d + 1]; e++) new_e += gcam_of[ecam[e]] < 0;
            if (d > c && ((int)gs.size() + new_s > gs_cap || (int)ge.size() + new_e > ge_cap))
                break;
            for (int s = P.ch_slot[d]; s < P.ch_slot[d + 1]; s++) {
                const int b = P.slot_blk[s];
                if (gslot_of[b] < 0) {
                    gslot_of[b] = (int)gs.size();
                    gs.push_back(b);
                }
                P.cs_g[s] = (unsigned short)gslot_of[b];
            }
            for (int e = P.ch_eslot[d]; e < P.ch_eslot[d + 1]; e++) {
                const int j = ecam[e];
                if (gcam_of[j] < 0) {
                    gcam_of[j] = (int)ge.size();
                    ge.push_back(j);
                }
                P.ce_g[e] = (unsigned short)gcam_of[j];
            }
            if ((int)gs.size() > gs_cap) {   // direct group: this chunk alone
                d++;
                break;
            }
        }
        for (int b : gs) {
            P.gslot_blk.push_back(b);
            gslot_of[b] = -1;
        }
        for (int j : ge) {
            P.gecam.push_back(j);
            gcam_of[j] = -1;
        }
        if (mf) {
            P.mf_max_s = std::max(P.mf_max_s, (int)gs.size());
            P.mf_max_e = std::max(P.mf_max_e, (int)ge.size());
            P.ngrp_mf++;
        } else if ((int)gs.size() <= gs_cap) {   // LDS accumulators actually needed
            P.grp_max_s = std::max(P.grp_max_s, (int)gs.size());
            P.grp_max_e = std::max(P.grp_max_e, (int)ge.size());
        }
        P.grp_ch.push_back(d);
        P.grp_gs.push_back((int)P.gslot_blk.size());
        P.grp_ge.push_back((int)P.gecam.size());
        c = d;
    }
    PLAN_T("groups");
    // long tracks' Schur terms (no slots of their own): k_schur_reduce adds,
    // per block (j, k), the terms Y_a W_b^T of every long track that sees both
    // cameras, in track order, by merging the two cameras' lists of long-track
    // observations (cam_lptr / cam_lobs / cam_ltrk: per camera its long-track
    // observations in ascending order = track order; a point sees a camera at
    // most once).  One group e-slot per long observation (its Y_a eB_i term,
    // k_long_y), after the regular ones.
    const int nlong = (int)P.long_pt.size();
    const int L0 = nlong ? P.long_o0[0] : 0, nlobs = nlong ? P.long_o0[nlong] - L0 : 0;
    for (int l = 0; l < nlong; l++)
        P.long_ebase.push_back((int)P.gecam.size() + (P.long_o0[l] - L0));
    P.gecam.insert(P.gecam.end(), lcam.begin() + L0, lcam.begin() + L0 + nlobs);
    {
        P.cam_lptr.assign(m + 1, 0);
        for (int o = L0; o < L0 + nlobs; o++) P.cam_lptr[lcam[o] + 1]++;
        for (int j = 0; j < m; j++) P.cam_lptr[j + 1] += P.cam_lptr[j];
        P.cam_lobs.resize(nlobs);
        P.cam_ltrk.resize(nlobs);
        std::vector<int> pos(P.cam_lptr.begin(), P.cam_lptr.end() - 1);
        for (int l = 0; l < nlong; l++)
            for (int o = P.long_o0[l]; o < P.long_o0[l + 1]; o++) {
                const int q = pos[lcam[o]]++;
                P.cam_lobs[q] = o - L0;
                P.cam_ltrk[q] = l;
            }
        for (int j = 0; j < m; j++)
            P.max_lcam = std::max(P.max_lcam, P.cam_lptr[j + 1] - P.cam_lptr[j]);
    }
    PLAN_T("long lists");
#ifdef BA_PLAN_TIMING
    std::fprintf(stderr, "   (group slots %zu; group e-slots %zu; long tracks %d, %d observations, "
                 "at most %d per camera)\n", P.gslot_blk.size(), P.gecam.size(), nlong, nlobs,
                 P.max_lcam);
#endif
    bucket(P.gslot_blk, nb, P.blk_gptr, P.blk_gslots);
    bucket(P.gecam, m, P.cam_gptr, P.cam_gslots);
    PLAN_T("buckets");
    P.ch_blob.assign(1, 0);
    P.ch_obase.assign(1, lptr[0]);
    if (P.nch_mf > 0) {
        // dense-layout record per chunk (k_schur_mfma):
        //   [np | nobs << 16]
        //   [C | flags << 8 | Kc << 16]  C cameras ascending, Kc = 3 np rounded to 4;
        //        flags: 1 dense (every point sees every camera of the chunk),
        //               2 flush (the next chunk of the group has other cameras, or
        //                 this is the group's last chunk: the register-held MFMA
        //                 tiles and e_ sums go to the group accumulators)
        //   ge[C]       group e-slot of each camera slot
        //   pair[C(C+1)/2]  group slot of block (cam[cr], cam[cc]), cr >= cc, index
        //                   cr (cr + 1) / 2 + cc; 0xffffffff: not in the group
        //   idx[ceil(np C / 4)]  byte p C + cs: local observation index of chunk
        //                        point p in camera slot cs, 0xff if p does not see it
        std::vector<int> cslot(m, -1), gsl_of(nb, -1), gel_of(m, -1);
        std::vector<int> ch_grp(nch);
        for (int g = 0; g + 1 < (int)P.grp_ch.size(); g++)
            for (int c = P.grp_ch[g]; c < P.grp_ch[g + 1]; c++) ch_grp[c] = g;
        auto cams_of = [&](int c, std::vector<int> &cams) {   // (reused buffers)
            cams.assign(ecam.begin() + P.ch_eslot[c], ecam.begin() + P.ch_eslot[c + 1]);
            std::sort(cams.begin(), cams.end());
        };
        std::vector<int> cams, next;
        std::vector<unsigned char> tab;
        cams_of(0, cams);
        for (int c = 0; c < P.nch_mf; c++) {
            const int g = ch_grp[c];
            if (c == P.grp_ch[g]) {   // group-local slot / camera ids
                for (int q = P.grp_gs[g]; q < P.grp_gs[g + 1]; q++)
                    gsl_of[P.gslot_blk[q]] = q - P.grp_gs[g];
                for (int q = P.grp_ge[g]; q < P.grp_ge[g + 1]; q++)
                    gel_of[P.gecam[q]] = q - P.grp_ge[g];
            }
            const int p0 = P.ch_pt[c], p1 = P.ch_pt[c + 1];
            const int nobs = lptr[p1] - lptr[p0];
            const int C = (int)cams.size();
            bool flush = true;
            next.clear();
            if (c + 1 < P.nch_mf) {
                cams_of(c + 1, next);
                flush = ch_grp[c + 1] != g || next != cams;
            }
            for (int q = 0; q < C; q++) cslot[cams[q]] = q;
            const bool dense = nobs == (p1 - p0) * C;
            std::vector<unsigned> &B = P.blob;
            const int kc = (3 * (p1 - p0) + 3) & ~3;
            B.push_back((unsigned)(p1 - p0) | ((unsigned)nobs << 16));
            B.push_back((unsigned)C | ((unsigned)(dense ? 1 : 0) << 8) |
                        ((unsigned)(flush ? 2 : 0) << 8) | ((unsigned)kc << 16));
            for (int q = 0; q < C; q++) B.push_back((unsigned)gel_of[cams[q]]);
            for (int cr = 0; cr < C; cr++)
                for (int cc = 0; cc <= cr; cc++) {
                    const int blk = hb.find(cams[cr], cams[cc]);
                    const int sl = blk >= 0 ? gsl_of[blk] : -1;
                    B.push_back(sl >= 0 ? (unsigned)sl : 0xffffffffu);
                }
            {
                tab.assign((size_t)(p1 - p0) * C, 0xff);
                for (int i = p0; i < p1; i++)
                    for (int o = lptr[i]; o < lptr[i + 1]; o++)
                        tab[(size_t)(i - p0) * C + cslot[lcam[o]]] =
                            (unsigned char)(o - lptr[p0]);
                for (size_t q = 0; q < tab.size(); q += 4) {
                    unsigned w = 0;
                    for (size_t u = 0; u < 4; u++)
                        w |= (unsigned)(q + u < tab.size() ? tab[q + u] : 0xff) << (8 * u);
                    B.push_back(w);
                }
            }
            for (int q = 0; q < C; q++) cslot[cams[q]] = -1;
            if (c + 1 == P.grp_ch[g + 1]) {
                for (int q = P.grp_gs[g]; q < P.grp_gs[g + 1]; q++) gsl_of[P.gslot_blk[q]] = -1;
                for (int q = P.grp_ge[g]; q < P.grp_ge[g + 1]; q++) gel_of[P.gecam[q]] = -1;
            }
            P.ch_blob.push_back((int)B.size());
            P.ch_obase.push_back(lptr[p1]);
            cams.swap(next);
        }
        for (int g = 0; g < P.ngrp_mf; g++)
            P.mf_max_blob = std::max(P.mf_max_blob,
                                     P.ch_blob[P.grp_ch[g + 1]] - P.ch_blob[P.grp_ch[g]]);
    }
    {   // term-chunk records: sizes first, then filled in parallel at their offsets
        const int nt = nch - P.nch_mf;
        std::vector<long long> boff(nt + 1, 0);
        for (int c = P.nch_mf; c < nch; c++) {
            const int s0 = P.ch_slot[c], s1 = P.ch_slot[c + 1];
            const int e0 = P.ch_eslot[c], e1 = P.ch_eslot[c + 1];
            const long long sz = 4 + (s1 - s0 + 1) + (e1 - e0 + 1) + (s1 - s0) + (e1 - e0) +
                                 (lptr[P.ch_pt[c + 1]] - lptr[P.ch_pt[c]]) +
                                 (P.slot_tptr[s1] - P.slot_tptr[s0]) +
                                 (P.eslot_optr[e1] - P.eslot_optr[e0]);
            boff[c - P.nch_mf + 1] = boff[c - P.nch_mf] + sz;
            P.ch_blob.push_back(P.ch_blob.back() + (int)sz);
            P.ch_obase.push_back(lptr[P.ch_pt[c + 1]]);
            P.max_blob = std::max(P.max_blob, (int)sz);
        }
        const size_t bbase = P.blob.size();
        P.blob.resize(bbase + boff[nt]);
        parallel_ranges(nt, plan_threads(boff[nt], 100000), [&](int, int c0, int c1) {
            for (int c = P.nch_mf + c0; c < P.nch_mf + c1; c++) {
                const int p0 = P.ch_pt[c], p1 = P.ch_pt[c + 1];
                const int nobs = lptr[p1] - lptr[p0];
                const int s0 = P.ch_slot[c], s1 = P.ch_slot[c + 1];
                const int e0 = P.ch_eslot[c], e1 = P.ch_eslot[c + 1];
                const int t0 = P.slot_tptr[s0], t1 = P.slot_tptr[s1];
                const int u0 = P.eslot_optr[e0], u1 = P.eslot_optr[e1];
                unsigned *B = &P.blob[bbase + boff[c - P.nch_mf]];
                *B++ = (unsigned)(p1 - p0) | ((unsigned)nobs << 16);
                *B++ = (unsigned)(s1 - s0) | ((unsigned)(e1 - e0) << 16);
                *B++ = (unsigned)(t1 - t0);
                *B++ = (unsigned)(u1 - u0);
                for (int s = s0; s <= s1; s++) *B++ = (unsigned)(P.slot_tptr[s] - t0);
                for (int e = e0; e <= e1; e++) *B++ = (unsigned)(P.eslot_optr[e] - u0);
                for (int s = s0; s < s1; s++) *B++ = P.cs_g[s];
                for (int e = e0; e < e1; e++) *B++ = P.ce_g[e];
                for (int i = p0; i < p1; i++)
                    for (int o = lptr[i]; o < lptr[i + 1]; o++) *B++ = (unsigned)(i - p0);
                for (int t = t0; t < t1; t++)
                    *B++ = (unsigned)P.slot_term[2 * t] | ((unsigned)P.slot_term[2 * t + 1] << 16);
                for (int u = u0; u < u1; u++) *B++ = P.eslot_obs[u];
            }
        }, &boff);
    }
    PLAN_T("blobs");
    for (size_t l = 0; l < P.long_pt.size(); l++)   // segment chunks: no Schur record
        for (int o = P.long_o0[l]; o < P.long_o0[l + 1]; o += BA_CH_OBS) {
            P.ch_blob.push_back(P.ch_blob.back());
            P.ch_obase.push_back(std::min(o + BA_CH_OBS, P.long_o0[l + 1]));
        }
    return true;
}

}  // namespace

void kt_begin(ba_ktimer *t, hipStream_t s)
{
    if (t->nev + 2 > KT_MAX_EV) return;
    while (t->ncreated < t->nev + 2) {
        if (hipEventCreate(&t->ev[t->ncreated]) != hipSuccess) return;   // (kt_end skips too)
        t->ncreated++;
    }
    (void)hipEventRecord(t->ev[t->nev], s);
}

void kt_end(ba_ktimer *t, hipStream_t s, int kid)
{
    if (t->nev + 2 > KT_MAX_EV || t->nev + 2 > t->ncreated) return;
    (void)hipEventRecord(t->ev[t->nev + 1], s);
    t->kid[t->nev / 2] = kid;
    t->nev += 2;
}

// =========================================================================
struct ba_aux {
    int device;
    hipStream_t stream, side;
    hipEvent_t ev_fork, ev_join;
    double *hres_host, *hres_dev;
    double *pin;        // pinned host staging of set_params (grown on demand)
    size_t pin_cap;     // its capacity in doubles
};

struct vlgba_ctx {
    ba_dev d;
    ba_flags flags;
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    int (*host_allreduce)(double *, long long, void *) = nullptr;
    void *host_user = nullptr;
    int p0 = 0, p1 = 0;          // global point range of this rank
    int n_global = 0;
    long long N_global = 0;
    double num_vis = 0;
    int max_iter = 20, max_iter2 = 10, verbose = 0;
    double lambda = 1e-3, lambda0 = 1e-3, nu = 2.0;
    int model = VLGBA_MODEL_EUCLIDEAN;
    int lin_valid = 0;
    int camred_due = 0;           // fused update: the linearisation swapped in by an
                                  // accepted step still needs its camera reduction
    int timing = 0;
    hipEvent_t ev[8] = {};
    double phase_ms[7] = {};
    std::vector<void *> allocs;
    std::vector<double> hb_tmp;   // host staging for b gather
    ba_aux aux;                   // streams / events / host result block (pooled)
    bool has_aux = false;
    double stop_rel = 1e-3;       // bundle_euclid.m:123 relative-decrease stop
    void (*on_pass)(int, int, const vlgba_step_info *, void *) = nullptr;
    void *on_pass_user = nullptr;
    // pinv fallback of the reduced solve (allocated on first use)
    // internal point order (fast path, one rank): the short-track points that
    // fit the MFMA Schur chunks first, then the rest, each in input order.
    // pperm[new] = input point, operm[new obs] = input observation (point-major
    // input order), both relative to this rank's first point / observation;
    // empty = identity.
    std::vector<int> pperm, operm;
    double *pinv_S = nullptr, *pinv_ev = nullptr, *pinv_e = nullptr, *pinv_w = nullptr;
    int *pinv_info = nullptr;
    int pinv_used = 0;            // passes that took the pinv fallback
    int nd_retries = 0;           // nested-dissection pivots solved in the natural order
    int spin_retries = 0;         // passes re-solved after a hand-off timeout
    int debug_timeouts = 0;       // test hooks: passes whose timeout word / pivot word
    int debug_pivots = 0;         // is forced (vlgba_debug_force_status)
};

// Per-device pool of the context's streams, fork/join events and host-mapped
// result block: creating them (pinned host memory above all) costs ~0.4 ms,
// which the growing-BA replay would pay per solve.  A context takes one set
// for its lifetime and returns it idle (both streams synchronised).
static std::mutex g_aux_mu;
static std::vector<ba_aux> g_aux_pool;

static int aux_acquire(int device, ba_aux &a)
{
    {
        std::lock_guard<std::mutex> lk(g_aux_mu);
        for (size_t q = 0; q < g_aux_pool.size(); q++)
            if (g_aux_pool[q].device == device) {
                a = g_aux_pool[q];
                g_aux_pool.erase(g_aux_pool.begin() + (long)q);
                a.hres_host[7] = 0.0;   // sequence numbers restart at 1
                return 0;
            }
    }
    std::memset(&a, 0, sizeof a);
    a.device = device;
    void *h = nullptr;
    if (hipStreamCreateWithFlags(&a.stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&a.side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&a.ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&a.ev_join, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&h, 8 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&a.hres_dev, h, 0) != hipSuccess) {
        if (a.stream) (void)hipStreamDestroy(a.stream);
        if (a.side) (void)hipStreamDestroy(a.side);
        if (a.ev_fork) (void)hipEventDestroy(a.ev_fork);
        if (a.ev_join) (void)hipEventDestroy(a.ev_join);
        if (h) (void)hipHostFree(h);
        return -1;
    }
    std::memset(h, 0, 8 * sizeof(double));
    a.hres_host = (double *)h;
    return 0;
}

static void aux_release(const ba_aux &a)
{
    (void)hipStreamSynchronize(a.stream);
    (void)hipStreamSynchronize(a.side);
    std::lock_guard<std::mutex> lk(g_aux_mu);
    g_aux_pool.push_back(a);
}

// RCCL communicators outlive their context, keyed by (unique id, world size,
// rank): a caller that passes the same id again (dist.run_sharded keeps one
// id per device set for a whole growing replay) takes the idle communicator
// instead of paying ncclCommInitRank per solve.  One context per key at a
// time.  An idle communicator is destroyed only when its caller says the id
// is done (vlgba_comm_release): a unique id serves ONE bootstrap, so evicting
// the communicator of an id the caller may pass again would send that next
// context into an ncclCommInitRank that waits forever.
struct comm_key {
    std::string id;
    int world, rank;
    bool operator<(const comm_key &o) const
    {
        if (id != o.id) return id < o.id;
        if (world != o.world) return world < o.world;
        return rank < o.rank;
    }
};
static std::mutex g_comm_mu;
static std::multimap<comm_key, ncclComm_t> g_comm_idle;
static std::map<ncclComm_t, comm_key> g_comm_key;

static ncclResult_t comm_acquire(ncclComm_t *comm, int world, const void *id128, int rank)
{
    const comm_key key{std::string((const char *)id128, 128), world, rank};
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        auto it = g_comm_idle.find(key);
        if (it != g_comm_idle.end()) {
            *comm = it->second;
            g_comm_idle.erase(it);
            return ncclSuccess;
        }
    }
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof id);
    const ncclResult_t r = ncclCommInitRank(comm, world, id, rank);
    if (r == ncclSuccess) {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        g_comm_key[*comm] = key;
    }
    return r;
}

// idle communicators kept at most (a caller that makes a fresh unique id per
// solve and never calls vlgba_comm_release would otherwise keep one per rank
// per solve for the life of the process): past the cap one idle communicator
// of another id is destroyed, with a warning the first time
#ifndef BA_COMM_IDLE_CAP
#define BA_COMM_IDLE_CAP 64
#endif

static void comm_release(ncclComm_t comm)
{
    ncclComm_t evict = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        auto it = g_comm_key.find(comm);
        if (it == g_comm_key.end()) {
            evict = comm;   // its id was released while this context held it
        } else {
            const comm_key key = it->second;
            g_comm_idle.emplace(key, comm);
            if (g_comm_idle.size() > BA_COMM_IDLE_CAP) {
                for (auto q = g_comm_idle.begin(); q != g_comm_idle.end(); ++q)
                    if (q->first < key || key < q->first) {
                        evict = q->second;
                        g_comm_key.erase(evict);
                        g_comm_idle.erase(q);
                        break;
                    }
                static bool warned = false;
                if (evict && !warned) {
                    warned = true;
                    std::fprintf(stderr, "[vlgba] more than %d idle RCCL communicators: "
                                         "destroying the oldest ids' (call vlgba_comm_release "
                                         "for ids that will not be used again)\n",
                                 BA_COMM_IDLE_CAP);
                }
            }
        }
    }
    if (evict) ncclCommDestroy(evict);
}

static void kt_retire(const ba_ktimer *kt);

static void ctx_free(vlgba_ctx *c)
{
    if (!c) return;
    if (c->d.stream) (void)hipStreamSynchronize(c->d.stream);
    if (c->d.side) (void)hipStreamSynchronize(c->d.side);
    for (void *p : c->allocs) ba_dfree(p);
    for (void *p : {(void *)c->pinv_S, (void *)c->pinv_ev, (void *)c->pinv_e, (void *)c->pinv_w,
                    (void *)c->pinv_info})
        if (p) ba_dfree(p);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->d.kt) {
        kt_retire(c->d.kt);
        for (int q = 0; q < c->d.kt->ncreated; q++) (void)hipEventDestroy(c->d.kt->ev[q]);
        delete c->d.kt;
    }
    ba_chol_free(&c->d);
    if (c->comm) comm_release(c->comm);
    if (c->has_aux) aux_release(c->aux);
    delete c;
}

template <typename T>
static int ctx_alloc(vlgba_ctx *c, T **p, size_t count)
{
    TRY(dalloc(p, count));
    c->allocs.push_back((void *)*p);
    return 0;
}

static int allreduce(vlgba_ctx *c, double *buf, size_t count)
{
    if ((c->world <= 1 && !c->comm) || count == 0) return 0;
    if (c->comm) {
        ncclResult_t r =
            ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c->comm, c->d.stream);
        return r == ncclSuccess ? 0 : VLGBA_E_COMM;
    }
    // host collective (vlgba_options.allreduce): device -> host, sum, host -> device
    c->hb_tmp.resize(count);
    TRY(download(c->hb_tmp.data(), buf, count, c->d.stream));
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    if (c->host_allreduce(c->hb_tmp.data(), (long long)count, c->host_user) != 0)
        return VLGBA_E_COMM;
    TRY(upload(buf, c->hb_tmp.data(), count, c->d.stream));
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    return 0;
}

// setup timing trace (VLGBA_SETUP_TRACE=1: one stderr line per context)
struct setup_trace {
    bool on = std::getenv("VLGBA_SETUP_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    std::string line;
    void mark(const char *what)
    {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        char buf[64];
        std::snprintf(buf, sizeof buf, " %s=%.0fus", what,
                      std::chrono::duration<double, std::micro>(now - t).count());
        line += buf;
        t = now;
    }
    ~setup_trace()
    {
        if (on && !line.empty()) std::fprintf(stderr, "[vlgba setup]%s\n", line.c_str());
    }
};
static thread_local setup_trace *g_st = nullptr;
#define ST_MARK(w) do { if (g_st) g_st->mark(w); } while (0)

// Fast-path point order by track kind (stable within a kind): short tracks
// (<= BA_MF_CMAX(na) views: MFMA Schur chunks) first, then tracks that fit a
// per-term chunk, then long tracks (split into chunk-sized segments with the
// dedicated long-track kernels), so that every kind is one contiguous range.
// Applied when more than one kind is present and no track exceeds the
// long-track caps (else the ordered kernels take the problem).  The
// summation order of the fast path changes with it (it is not the parity
// path); set / get_params and the getters map back to the input order.
static int track_kind(long long k, int cmax)
{
    if (k <= cmax) return 0;                                      // MFMA Schur chunk
    if (k <= BA_CH_OBS && k * (k + 1) / 2 <= BA_CH_TERMS) return 1;   // per-term chunk
    return 2;                                                     // long track
}

static void order_points_by_kind(int cmax, host_obs &h, std::vector<int> &pt_ptr, int p0,
                                 int p1, std::vector<int> &pperm, std::vector<int> &operm)
{
    // points [p0, p1) of the global point-major arrays (this rank's range);
    // pperm / operm are relative to p0 / the range's first observation
    const int n = p1 - p0;
    int cnt[3] = {0, 0, 0};
    long long lterms = 0;
    for (int i = p0; i < p1; i++) {
        const long long k = pt_ptr[i + 1] - pt_ptr[i];
        const int kind = track_kind(k, cmax);
        cnt[kind]++;
        if (kind == 2) {
            if (k > BA_LONG_OBS) return;                          // ordered kernels
            lterms += k * (k + 1) / 2;
        }
    }
    if (lterms > BA_LONG_TERMS) return;
    if ((cnt[0] == 0) + (cnt[1] == 0) + (cnt[2] == 0) >= 2) return;   // one kind: as is
    // stable placement by kind (one counting pass instead of three scans)
    pperm.assign(n, 0);
    {
        int at[3] = {0, cnt[0], cnt[0] + cnt[1]};
        for (int i = 0; i < n; i++) pperm[at[track_kind(pt_ptr[p0 + i + 1] - pt_ptr[p0 + i], cmax)]++] = i;
    }
    const int o0 = pt_ptr[p0];
    const size_t N = (size_t)(pt_ptr[p1] - o0);
    std::vector<int> cam2(N);
    std::vector<double> x2(2 * N);
    operm.resize(N);
    std::vector<int> ptr2(n + 1, 0);
    size_t q = 0;
    for (int i2 = 0; i2 < n; i2++) {
        const int i = p0 + pperm[i2];
        for (int o = pt_ptr[i]; o < pt_ptr[i + 1]; o++, q++) {
            cam2[q] = h.cam[o];
            x2[2 * q] = h.x[2 * (size_t)o];
            x2[2 * q + 1] = h.x[2 * (size_t)o + 1];
            operm[q] = o - o0;
        }
        ptr2[i2 + 1] = (int)q;
    }
    if (o0 == 0 && N == h.cam.size()) {   // the whole list (one rank): swap, no copy back
        h.cam.swap(cam2);
        h.x.swap(x2);
    } else {
        std::copy(cam2.begin(), cam2.end(), h.cam.begin() + o0);
        std::copy(x2.begin(), x2.end(), h.x.begin() + 2 * (size_t)o0);
    }
    for (int i2 = 0; i2 < n; i2++) {
        pt_ptr[p0 + i2 + 1] = o0 + ptr2[i2 + 1];
        for (int o = ptr2[i2]; o < ptr2[i2 + 1]; o++) h.pt[o0 + o] = p0 + i2;
    }
}

// The host side of a context's plan (ctx_setup; tools/bench_plan.cpp times it
// on the CPU): the co-visible block set and, on the fast path, the chunk /
// group plan.  fast is cleared when some track fits no chunk kind (the
// ordered kernels take the problem; hb then carries their term lists).
static void plan_host(int m, int na, int n, const std::vector<int> &lptr,
                      const std::vector<int> &lcam, const std::vector<int> &pt_ptr_all,
                      const std::vector<int> &cam_all, int p0, int p1, long long o0,
                      bool lower_blocks, bool all_diag, bool no_mfma, bool &fast, int &p_long,
                      host_blocks &hb, host_plan &plan)
{
    // long tracks (more than a chunk holds) must form the tail [p_long, n) of
    // the local points (order_points_by_kind) and stay within the caps; else
    // the sequential kernels take the problem
    p_long = n;
    if (fast) {
        while (p_long > 0 && track_kind(lptr[p_long] - lptr[p_long - 1], BA_MF_CMAX(na)) == 2)
            p_long--;
        long long lterms = 0;
        for (int i = 0; fast && i < n; i++) {
            const long long k = lptr[i + 1] - lptr[i];
            const bool lng = track_kind(k, BA_MF_CMAX(na)) == 2;
            if (lng != (i >= p_long) || k > BA_LONG_OBS) fast = false;
            if (lng) lterms += k * (k + 1) / 2;
        }
        if (lterms > BA_LONG_TERMS) fast = false;
    }
    build_blocks(m, pt_ptr_all, cam_all, p0, p1, o0, lower_blocks, all_diag, !fast, hb);
    ST_MARK("blocks");
    // MFMA Schur chunks for the leading points whose tracks fit the dense slab
    // (ctx_create orders the short-track points first), per-term chunks for
    // the rest; the ordered kernels if some track fits neither
    if (fast) {
        int p_split = 0;
        if (!no_mfma)
            while (p_split < p_long && lptr[p_split + 1] - lptr[p_split] <= BA_MF_CMAX(na))
                p_split++;
        if (!build_plan(m, na, lptr, lcam, hb, plan, BA_MF_CMAX(na), p_split, p_long)) {
            fast = false;
            hb = host_blocks();
            build_blocks(m, pt_ptr_all, cam_all, p0, p1, o0, lower_blocks, all_diag, true, hb);
        }
    }
}

// A context's plan arrays (~30 host vectors) go to the device as ONE copy:
// each array at a 256-byte aligned offset of one device block and of the
// context's pinned staging buffer (ba_aux::pin, which set_params reuses) --
// one hipMemcpyAsync from pinned memory instead of one pageable copy per
// array (the setup trace's plan_upload: 1.1 ms per context over the growing
// replay, profiles/r06/r06f_cfg5x_setup_phases.txt).  The pointers stay valid
// for the context's life (the block is one of its allocations).
struct plan_batch {
    struct item {
        void **dst;
        const void *src;
        size_t bytes, off;
    };
    std::vector<item> items;
    size_t total = 0;
    template <typename T> void add(T **dst, const std::vector<T> &v)
    {
        items.push_back({(void **)dst, v.data(), sizeof(T) * v.size(), total});
        total += (sizeof(T) * std::max<size_t>(v.size(), 1) + 255) & ~(size_t)255;
    }
    int commit(vlgba_ctx *c, hipStream_t s)
    {
        if (items.empty()) return 0;
        char *dev = nullptr;
        TRY(ctx_alloc(c, &dev, total));
        ba_aux &x = c->aux;
        const size_t need = (total + sizeof(double) - 1) / sizeof(double);
        if (x.pin_cap < need) {
            if (x.pin) (void)hipHostFree(x.pin);
            size_t cap = 1 << 16;
            while (cap < need) cap <<= 1;
            x.pin = nullptr;
            x.pin_cap = 0;
            if (hipHostMalloc((void **)&x.pin, sizeof(double) * cap, hipHostMallocDefault) ==
                hipSuccess)
                x.pin_cap = cap;
        }
        char *stage = x.pin_cap >= need ? (char *)x.pin : nullptr;
        for (const item &it : items) {
            *it.dst = dev + it.off;
            if (it.bytes == 0) continue;
            if (stage)
                std::memcpy(stage + it.off, it.src, it.bytes);
            else   // (no pinned memory: array by array)
                VLGBA_CHECK(hipMemcpyAsync(dev + it.off, it.src, it.bytes,
                                           hipMemcpyHostToDevice, s));
        }
        if (stage)
            VLGBA_CHECK(hipMemcpyAsync(dev, stage, total, hipMemcpyHostToDevice, s));
        VLGBA_CHECK(hipStreamSynchronize(s));
        return 0;
    }
};

// Device buffers + host-side structure for the observations of points [p0, p1).
static int ctx_setup(vlgba_ctx *c, const vlgba_problem *p, const host_obs &h,
                     const std::vector<int> &pt_ptr_all, bool lower_blocks, bool all_diag,
                     bool stage_mode)
{
    ba_dev &d = c->d;
    const int na = p->num_a;
    d.device = c->aux.device;
    VLGBA_CHECK(hipDeviceGetAttribute(&d.ncu, hipDeviceAttributeMultiprocessorCount, d.device));
    d.m = p->m;
    d.na = na;
    d.js = 2 * na + 2;
    d.n = c->p1 - c->p0;
    const long long o0 = pt_ptr_all[c->p0], o1 = pt_ptr_all[c->p1];
    d.N = (int)(o1 - o0);
    d.ld = (long long)na * p->m;
    d.lds = ((d.ld + 63) / 64) * 64;
    // every rank adds its own partial U* / eA into its partial reduced system
    // (the damping is linear: sum_r (1 + lambda) U_r = (1 + lambda) sum_r U_r),
    // so U / eA never need an all-reduce of their own; the camera part of
    // dp'(lambda dp + g) takes its lambda dp'dp term from rank 0 only
    d.schur_owner = 1;
    d.dpg_lambda = c->rank == 0;
    hipStream_t s = d.stream;

    // local point-major arrays
    std::vector<int> lptr(d.n + 1), lcam(h.cam.begin() + o0, h.cam.begin() + o1);
    for (int i = 0; i <= d.n; i++) lptr[i] = pt_ptr_all[c->p0 + i] - (int)o0;
    // camera-major view of the local observations (obs ids ascending per camera)
    std::vector<int> cptr(p->m + 1, 0), cobs(d.N);
    for (int o = 0; o < d.N; o++) cptr[lcam[o] + 1]++;
    for (int j = 0; j < p->m; j++) cptr[j + 1] += cptr[j];
    {
        std::vector<int> pos(cptr.begin(), cptr.end() - 1);
        for (int o = 0; o < d.N; o++) cobs[pos[lcam[o]]++] = o;
    }
    bool fast = !d.ordered && !stage_mode;
    int p_long = d.n;
    // the host plan in this thread's scratch: its storage is kept from one
    // context to the next (the growing replay creates one per solve on its two
    // prefetch workers)
    static thread_local host_blocks hb;
    static thread_local host_plan plan;
    hb.reset();
    plan.reset();
    ST_MARK("lists");
    plan_host(p->m, na, d.n, lptr, lcam, pt_ptr_all, h.cam, c->p0, c->p1, o0, lower_blocks,
              all_diag, d.no_mfma != 0, fast, p_long, hb, plan);
    d.mfma = fast && plan.nch_mf > 0;
    if (!fast) d.ordered = 1;
    ST_MARK("plan");
    d.nb = (int)hb.jk.size() / 2;
    d.T = (long long)hb.term.size() / 2;

    TRY(ctx_alloc(c, &d.obs_cam, d.N));
    TRY(ctx_alloc(c, &d.pt_ptr, d.n + 1));
    TRY(ctx_alloc(c, &d.cam_ptr, p->m + 1));
    TRY(ctx_alloc(c, &d.cam_obs, d.N));
    TRY(ctx_alloc(c, &d.obs_x, 2 * (size_t)d.N));
    TRY(ctx_alloc(c, &d.K4, 4 * (size_t)p->m));
    TRY(ctx_alloc(c, &d.a, (size_t)d.ld));
    TRY(ctx_alloc(c, &d.a_new, (size_t)d.ld));
    TRY(ctx_alloc(c, &d.b, 3 * (size_t)d.n));
    TRY(ctx_alloc(c, &d.b_new, 3 * (size_t)d.n));
    TRY(ctx_alloc(c, &d.rot, 45 * (size_t)p->m));
    TRY(ctx_alloc(c, &d.rot_new, 45 * (size_t)p->m));
    // W, eB, V*^-1 carry one zero row past the end: the MFMA Schur kernel points
    // the fragment loads of absent (point, camera) pairs at it
    TRY(ctx_alloc(c, &d.W, (size_t)3 * na * (d.N + 1)));
    VLGBA_CHECK(hipMemsetAsync(d.W + (size_t)3 * na * d.N, 0, sizeof(double) * 3 * na, s));
    if (!fast) {   // the fast path forms A, e, Y and t in LDS only
        TRY(ctx_alloc(c, &d.jrec, (size_t)d.js * d.N));
        TRY(ctx_alloc(c, &d.Y, (size_t)3 * na * d.N));
        TRY(ctx_alloc(c, &d.t, (size_t)na * d.N));
    } else {
        d.nch_reg = plan.nch_reg;
        d.nch = plan.nch_reg + plan.nseg;
        d.nl = (int)plan.long_pt.size();
        d.max_lcam = plan.max_lcam;
        d.long_o0_h = plan.long_o0.empty() ? 0 : plan.long_o0[0];
        d.p_long = p_long;
        // the plan's arrays: one device block, one copy (plan_batch)
        plan_batch pb;
        if (d.nl > 0) {
            pb.add(&d.seg_pt, plan.seg_pt);
            pb.add(&d.seg_long, plan.seg_long);
            pb.add(&d.long_pt, plan.long_pt);
            pb.add(&d.long_o0, plan.long_o0);
            pb.add(&d.long_seg0, plan.long_seg0);
            pb.add(&d.long_ebase, plan.long_ebase);
            pb.add(&d.cam_lptr, plan.cam_lptr);
            pb.add(&d.cam_lobs, plan.cam_lobs);
            pb.add(&d.cam_ltrk, plan.cam_ltrk);
            TRY(ctx_alloc(c, &d.ylong, (size_t)3 * na * plan.cam_lobs.size()));
            TRY(ctx_alloc(c, &d.vseg, 12 * (size_t)plan.nseg));
            TRY(ctx_alloc(c, &d.dpg_long, (size_t)d.nl));
        }
        d.ns = (int)plan.slot_blk.size();
        d.nes = (int)plan.eslot_optr.size() - 1;
        d.ch_max_terms = plan.max_terms;
        d.ch_max_slots = plan.max_slots;
        d.nterm_fast = plan.n_terms;
        d.blob_words = (long long)plan.blob.size();
        d.ngrp = (int)plan.grp_ch.size() - 1;
        d.ngrp_mf = plan.ngrp_mf;
        d.max_blob = plan.max_blob;
        d.mf_max_blob = plan.mf_max_blob;
        d.mf_max_s = plan.mf_max_s;
        d.mf_max_e = plan.mf_max_e;
        pb.add(&d.blob, plan.blob);
        pb.add(&d.ch_blob, plan.ch_blob);
        pb.add(&d.ch_obase, plan.ch_obase);
        // chunk-local point of every observation (k_linearize_chunk) and each
        // chunk's camera range (k_update_linearize's da staging)
        std::vector<unsigned char> lpt(d.N > 0 ? d.N : 1, 0);
        for (size_t ch = 0; ch + 1 < plan.ch_pt.size(); ch++)
            for (int i = plan.ch_pt[ch]; i < plan.ch_pt[ch + 1]; i++)
                for (int o = lptr[i]; o < lptr[i + 1]; o++)
                    lpt[o] = (unsigned char)(i - plan.ch_pt[ch]);
        const size_t nchk = plan.ch_obase.size() - 1;
        std::vector<int> ccam(2 * std::max<size_t>(nchk, 1), 0);
        for (size_t ch = 0; ch < nchk; ch++) {
            int lo = INT_MAX, hi = -1;
            for (int o = plan.ch_obase[ch]; o < plan.ch_obase[ch + 1]; o++) {
                lo = std::min(lo, lcam[o]);
                hi = std::max(hi, lcam[o]);
            }
            ccam[2 * ch] = hi < 0 ? 0 : lo;
            ccam[2 * ch + 1] = hi < 0 ? 0 : hi;
        }
        // VLGBA_DA_STAGE=0 (A/B): every range too wide, each lane loads its da row
        const char *dse = std::getenv("VLGBA_DA_STAGE");
        if (dse && dse[0] == '0')
            for (size_t ch = 0; ch < nchk; ch++) ccam[2 * ch + 1] = ccam[2 * ch] + (1 << 20);
        pb.add(&d.obs_lpt, lpt);
        pb.add(&d.ch_cam, ccam);
        d.grp_max_s = plan.grp_max_s;
        d.grp_max_e = plan.grp_max_e;
        d.ngs = (int)plan.gslot_blk.size();
        d.nge = (int)plan.gecam.size();
        TRY(ctx_alloc(c, &d.spart, (size_t)na * na * d.ngs));
        TRY(ctx_alloc(c, &d.epart, (size_t)na * d.nge));
        pb.add(&d.grp_ch, plan.grp_ch);
        pb.add(&d.grp_gs, plan.grp_gs);
        pb.add(&d.grp_ge, plan.grp_ge);
        pb.add(&d.cs_g, plan.cs_g);
        pb.add(&d.ce_g, plan.ce_g);
        pb.add(&d.blk_gptr, plan.blk_gptr);
        pb.add(&d.blk_gslots, plan.blk_gslots);
        pb.add(&d.cam_gptr, plan.cam_gptr);
        pb.add(&d.cam_gslots, plan.cam_gslots);
        TRY(ctx_alloc(c, &d.upart, (size_t)(na * (na + 1) / 2 + na) * d.nes));
        TRY(ctx_alloc(c, &d.chsse, 3 * (size_t)d.nch));   // lin SSE | new SSE | dpg
        pb.add(&d.ch_pt, plan.ch_pt);
        pb.add(&d.ch_eslot, plan.ch_eslot);
        pb.add(&d.eslot_optr, plan.eslot_optr);
        pb.add(&d.eslot_obs, plan.eslot_obs);
        pb.add(&d.cam_eptr, plan.cam_eptr);
        pb.add(&d.cam_eslots, plan.cam_eslots);
        TRY(pb.commit(c, s));   // (synchronous: the plan vectors are thread scratch)
        ST_MARK("plan_upload");
    }
    TRY(ctx_alloc(c, &d.U, (size_t)na * na * p->m + na * (size_t)p->m + 1));
    d.eA = d.U + (size_t)na * na * p->m;     // U | eA | old_sse contiguous: one all-reduce
    TRY(ctx_alloc(c, &d.V, 9 * (size_t)d.n));
    TRY(ctx_alloc(c, &d.eB, 3 * (size_t)(d.n + 1)));
    TRY(ctx_alloc(c, &d.Vinv, 9 * (size_t)(d.n + 1)));
    VLGBA_CHECK(hipMemsetAsync(d.eB + 3 * (size_t)d.n, 0, sizeof(double) * 3, s));
    VLGBA_CHECK(hipMemsetAsync(d.Vinv + 9 * (size_t)d.n, 0, sizeof(double) * 9, s));
    TRY(ctx_alloc(c, &d.db, 3 * (size_t)d.n));
    // fused update (fast path): the next linearisation's buffers (VLGBA_FUSED=0
    // keeps the separate update and linearisation launches: A/B)
    const char *fused_env = std::getenv("VLGBA_FUSED");   // read per context (tests)
    const bool fused_on = !(fused_env && fused_env[0] == '0');
    if (fast && d.nch > 0 && fused_on) {
        TRY(ctx_alloc(c, &d.W2, (size_t)3 * na * (d.N + 1)));
        VLGBA_CHECK(hipMemsetAsync(d.W2 + (size_t)3 * na * d.N, 0, sizeof(double) * 3 * na, s));
        TRY(ctx_alloc(c, &d.V2, 9 * (size_t)d.n));
        TRY(ctx_alloc(c, &d.eB2, 3 * (size_t)(d.n + 1)));
        VLGBA_CHECK(hipMemsetAsync(d.eB2 + 3 * (size_t)d.n, 0, sizeof(double) * 3, s));
        TRY(ctx_alloc(c, &d.upart2, (size_t)(na * (na + 1) / 2 + na) * d.nes));
        TRY(ctx_alloc(c, &d.chsse2, 3 * (size_t)d.nch));
        d.fused = 1;
    }
    TRY(ctx_alloc(c, &d.blk_jk, 2 * (size_t)d.nb));
    TRY(ctx_alloc(c, &d.blk_ptr, (size_t)d.nb + 1));
    TRY(ctx_alloc(c, &d.term, 2 * (size_t)d.T));
    TRY(upload(d.blk_jk, hb.jk.data(), hb.jk.size(), s));
    // the long tracks' pair counts per block (k_long_pairs) on the device while
    // the host builds the solve's structure (ba_chol_setup); read back below
    int *lp_cnt = nullptr;
    if (fast && d.nl > 0) {
        TRY(ctx_alloc(c, &lp_cnt, (size_t)d.nb + 1));
        TRY(ctx_alloc(c, &d.lpair_ptr, (size_t)d.nb + 1));
        TRY(ba_launch_long_pairs(&d, 0, lp_cnt));
    }
    // blocks | rhs | old SSE contiguous: one all-reduce per pass (world > 1)
    TRY(ctx_alloc(c, &d.sblk, (size_t)na * na * d.nb + d.lds + 1));
    d.rhs = d.sblk + (size_t)na * na * d.nb;
    if (!stage_mode) {
        TRY(ctx_alloc(c, &d.da, (size_t)d.lds));   // S, linv, ywork: ba_chol_setup
        ST_MARK("allocs");
        TRY(ba_chol_setup(&d, hb.jk.data(), d.nb));
        ST_MARK("chol_setup");
        // direct assembly (ba_dev::asm_direct): one rank without a collective
        // between the block sums and the solve, the fast path's block sums, no
        // long tracks (k_schur_long_acc adds to the sums after them);
        // VLGBA_ASM_DIRECT=0 keeps k_assemble_tiles (A/B)
        const char *ad = std::getenv("VLGBA_ASM_DIRECT");
        d.asm_direct = d.asm_direct_ok && !(ad && ad[0] == '0') && fast && !d.ordered &&
                       c->world == 1 && !c->comm && d.nl == 0 && d.cr_nlev > 0 && d.cr32 &&
                       d.nd_np == 0;
    } else {
        TRY(ctx_alloc(c, &d.da, (size_t)d.lds));
    }
    TRY(ctx_alloc(c, &d.part, 3 * (size_t)BA_PART_MAX));
    TRY(ctx_alloc(c, &d.scal, 8));
    if (p->num_obs > 0 || true) {
        TRY(upload(d.obs_cam, lcam.data(), d.N, s));
        TRY(upload(d.pt_ptr, lptr.data(), d.n + 1, s));
        TRY(upload(d.cam_ptr, cptr.data(), p->m + 1, s));
        TRY(upload(d.cam_obs, cobs.data(), d.N, s));
        TRY(upload(d.obs_x, h.x.data() + 2 * o0, 2 * (size_t)d.N, s));
        if (p->K) TRY(upload(d.K4, p->K, 4 * (size_t)p->m, s));
        else VLGBA_CHECK(hipMemsetAsync(d.K4, 0, sizeof(double) * 4 * p->m, s));
        TRY(upload(d.blk_ptr, hb.ptr.data(), hb.ptr.size(), s));
        TRY(upload(d.term, hb.term.data(), hb.term.size(), s));
    }
    ST_MARK("uploads");
    if (fast && d.nl > 0) {   // the long tracks' per-block pair lists (k_long_pairs)
        std::vector<int> h((size_t)d.nb + 1, 0);
        TRY(download(h.data(), lp_cnt, (size_t)d.nb, s));
        VLGBA_CHECK(hipStreamSynchronize(s));
        long long tot = 0;
        for (int b = 0; b < d.nb; b++) {
            const int v = h[b];
            h[b] = (int)tot;
            tot += v;
        }
        h[d.nb] = (int)tot;
        if (tot > 0x7fffffffLL) return VLGBA_E_ARG;
        TRY(ctx_alloc(c, &d.lpair, (size_t)tot + 1));
        TRY(upload(d.lpair_ptr, h.data(), (size_t)d.nb + 1, s));
        TRY(ba_launch_long_pairs(&d, 1, nullptr));
        // the blocks with pairs for k_schur_long_acc, most pairs first
        // (VLGBA_LONG_ACC=0: k_schur_reduce streams them itself)
        const char *la = std::getenv("VLGBA_LONG_ACC");
        if (!(la && la[0] == '0')) {
            std::vector<int> lb;
            for (int b = 0; b < d.nb; b++)
                if (h[b + 1] > h[b]) lb.push_back(b);
            std::stable_sort(lb.begin(), lb.end(), [&](int x, int y) {
                return h[x + 1] - h[x] > h[y + 1] - h[y];
            });
            d.nlb = (int)lb.size();
            if (d.nlb > 0) {
                TRY(ctx_alloc(c, &d.lblk, lb.size()));
                TRY(upload(d.lblk, lb.data(), lb.size(), s));
            }
        }
        ST_MARK("long_pairs");
    }
    VLGBA_CHECK(hipMemsetAsync(d.scal, 0, 8 * sizeof(double), s));
    TRY(ctx_alloc(c, &d.pub_cnt, 1));
    VLGBA_CHECK(hipMemsetAsync(d.pub_cnt, 0, sizeof(unsigned), s));
    VLGBA_CHECK(hipStreamSynchronize(s));   // host vectors go out of scope
    return 0;
}

static int ctx_create(const vlgba_problem *p, const vlgba_options *o, vlgba_ctx **out,
                      bool lower_blocks, bool all_diag, bool stage_mode,
                      std::vector<int> *pt_ptr_out = nullptr, host_obs *h_out = nullptr)
{
    *out = nullptr;
    if (!p || p->m < 1 || p->n < 0 || p->num_obs < 0) return VLGBA_E_ARG;
    if (p->model == VLGBA_MODEL_EUCLIDEAN) {
        if (!p->K) return VLGBA_E_ARG;
        if (p->num_a != 6 && p->num_a != 7 && p->num_a != 10) return VLGBA_E_NUMA;
    } else if (p->model == VLGBA_MODEL_PROJECTIVE) {
        if (p->num_a != BA_PROJ_NA) return VLGBA_E_NUMA;
    } else {
        return VLGBA_E_ARG;
    }
    if (p->num_obs > 0x7fffffffLL) return VLGBA_E_ARG;
    vlgba_ctx *c = new (std::nothrow) vlgba_ctx();
    if (!c) return VLGBA_E_NOMEM;
    std::memset(&c->d, 0, sizeof(c->d));
    vlgba_options defaults;
    std::memset(&defaults, 0, sizeof defaults);
    if (!o) o = &defaults;
    int rc = 0;
    setup_trace trace;
    g_st = &trace;
    struct st_reset { ~st_reset() { g_st = nullptr; } } st_reset_;
    do {
        if (hipSetDevice(o->device) != hipSuccess) { rc = VLGBA_E_ARG; break; }
        if (aux_acquire(o->device, c->aux)) {
            rc = -1;
            break;
        }
        c->has_aux = true;
        c->d.stream = c->aux.stream;
        c->d.side = c->aux.side;
        c->d.ev_fork = c->aux.ev_fork;
        c->d.ev_join = c->aux.ev_join;
        c->d.hres = c->aux.hres_host;
        c->d.hres_dev = c->aux.hres_dev;
        ST_MARK("aux");
        host_obs h;
        rc = sort_obs(p, h);
        if (rc) break;
        ST_MARK("sort");
        std::vector<int> pt_ptr_all(p->n + 1, 0);
        for (size_t q = 0; q < h.pt.size(); q++) pt_ptr_all[h.pt[q] + 1]++;
        for (int i = 0; i < p->n; i++) pt_ptr_all[i + 1] += pt_ptr_all[i];
        c->world = o->world_size > 1 ? o->world_size : 1;
        c->rank = c->world > 1 ? o->rank : 0;
        // contiguous point ranges with balanced observation counts
        if (c->world > 1) {
            const long long N = p->num_obs;
            auto bound = [&](int r) -> int {
                const long long target = (N * r) / c->world;
                return (int)(std::lower_bound(pt_ptr_all.begin(), pt_ptr_all.end(), (int)target) -
                             pt_ptr_all.begin());
            };
            c->p0 = c->rank == 0 ? 0 : std::min(bound(c->rank), p->n);
            c->p1 = c->rank == c->world - 1 ? p->n : std::min(bound(c->rank + 1), p->n);
            if (o->comm_id) {
                if (comm_acquire(&c->comm, c->world, o->comm_id, c->rank) != ncclSuccess) {
                    rc = VLGBA_E_COMM;
                    break;
                }
            } else if (o->allreduce) {
                c->host_allreduce = o->allreduce;
                c->host_user = o->allreduce_user;
            } else {
                rc = VLGBA_E_COMM;
                break;
            }
        } else {
            c->p0 = 0;
            c->p1 = p->n;
            if (o->comm_id) {   // a one-rank RCCL communicator: every collective
                                // of the pass runs through RCCL (identity sums)
                if (comm_acquire(&c->comm, 1, o->comm_id, 0) != ncclSuccess) {
                    rc = VLGBA_E_COMM;
                    break;
                }
            }
        }
        // fast path: this rank's points by track kind (short tracks for the MFMA
        // Schur chunks first, per-term tracks, long tracks last); the ranges
        // of the other ranks are left as they are (the block set, the only
        // global structure a rank builds, is order independent: build_blocks)
        if (o->ordered == 0 && !stage_mode)
            order_points_by_kind(o->schur_kernel == 1 ? 0 : BA_MF_CMAX(p->num_a), h, pt_ptr_all,
                                 c->p0, c->p1, c->pperm, c->operm);
        ST_MARK("order");
        c->n_global = p->n;
        c->N_global = p->num_obs;
        c->num_vis = p->num_vis > 0 ? p->num_vis : (double)p->num_obs;
        c->flags.fix_structure = o->fix_structure;
        c->flags.fix_motion = o->fix_motion;
        if (o->semantics != 0 && o->semantics != 1) { rc = VLGBA_E_ARG; break; }
        // bundle_euclid_nomex.m has no fix_pivot option: the pivot is ignored there
        // (nor has bundle_projective.m, :46-56)
        c->flags.has_pivot = o->pivot != nullptr && o->semantics == 0 &&
                             p->model == VLGBA_MODEL_EUCLIDEAN;
        c->model = p->model;
        c->max_iter = o->max_iter > 0 ? o->max_iter : 20;
        c->max_iter2 = o->max_iter2 > 0 ? o->max_iter2 : 10;
        c->lambda0 = c->lambda = o->lambda0 > 0 ? o->lambda0 : 1e-3;
        c->verbose = o->verbose;
        c->d.dense_solve = o->dense_solve;
        c->d.ordered = o->ordered != 0;
        if (o->ordered == 2) {   // parity mode: + sequential solve and LM scalars
            if (c->world > 1) { rc = VLGBA_E_ARG; break; }
            c->d.parity = 1;
            c->d.dense_solve = 3;
        } else if (o->ordered < 0 || o->ordered > 2 || o->dense_solve < 0 ||
                   o->dense_solve > 4) {
            rc = VLGBA_E_ARG;
            break;
        }
        c->stop_rel = o->stop_rel > 0 ? o->stop_rel : 1e-3;
        if (const char *ev = std::getenv("VLGBA_DEBUG_SPIN_TIMEOUT")) {
            // "R:K": rank R's first K passes report a hand-off timeout (tests)
            int r = -1, k = 0;
            if (std::sscanf(ev, "%d:%d", &r, &k) == 2 && r == c->rank) c->debug_timeouts = k;
            // a leftover variable would silently force re-solves: say so
            if (c->debug_timeouts > 0)
                std::fprintf(stderr, "[vlgba] VLGBA_DEBUG_SPIN_TIMEOUT=%s: rank %d's first %d "
                             "passes report a hand-off timeout (test hook)\n", ev, r, k);
        }
        c->on_pass = o->on_pass;
        c->on_pass_user = o->on_pass_user;
        c->d.no_mfma = o->schur_kernel == 1;
        c->d.fuse_camred = BA_FUSE_CAMRED;
        c->d.ndb = o->semantics == 1 ? p->num_a : 6;
        rc = ctx_setup(c, p, h, pt_ptr_all, lower_blocks, all_diag, stage_mode);
        if (rc) break;
        ST_MARK("setup_end");
        if (c->d.parity) {   // new projections for the sequential new-SSE sum
            rc = ctx_alloc(c, &c->d.xh_out, 2 * (size_t)c->d.N + 2);
            if (rc) break;
        }
        if (c->flags.has_pivot) {
            rc = ctx_alloc(c, &c->d.pivot, (size_t)p->m);
            if (rc) break;
            rc = upload(c->d.pivot, o->pivot, (size_t)p->m, c->d.stream);
            if (rc) break;
        }
        if (std::getenv("VLGBA_KTIME_ALL")) {   // every context times its passes
            rc = vlgba_set_timing(c, 1);
            if (rc) break;
        }
        if (pt_ptr_out) *pt_ptr_out = pt_ptr_all;
        if (h_out) *h_out = std::move(h);
    } while (0);
    if (rc) {
        ctx_free(c);
        return rc;
    }
    *out = c;
    return 0;
}

// ---------------------------------------------------------------------------
// one LM pass
// ---------------------------------------------------------------------------
static inline void mark(vlgba_ctx *c, int q)
{
    if (c->timing) (void)hipEventRecord(c->ev[q], c->d.stream);
}

// damping + V*^-1 + Y + Schur complement (S blocks, e_) and their all-reduce
static int schur_phase(vlgba_ctx *c, double lam)
{
    ba_dev &d = c->d;
    mark(c, 2);
    if (d.ordered) {
        TRY(ba_launch_damp_point(&d, lam));
        mark(c, 3);
        TRY(ba_launch_schur(&d, lam));
    } else {
        mark(c, 3);
        TRY(ba_launch_schur_fast(&d, lam));
    }
    if (c->world > 1 || c->comm) {
        // [S blocks | e_ | old SSE] of this rank's points -> the global system
        double *sse = d.rhs + d.lds;
        VLGBA_CHECK(hipMemcpyAsync(sse, d.eA + d.ld, sizeof(double), hipMemcpyDeviceToDevice,
                                   d.stream));
        TRY(allreduce(c, d.sblk, (size_t)d.na * d.na * d.nb + d.lds + 1));
        VLGBA_CHECK(hipMemcpyAsync(d.scal + 0, sse, sizeof(double), hipMemcpyDeviceToDevice,
                                   d.stream));
    }
    return 0;
}

// the pass scalars after the update: cross-rank sums, then to the host (spin
// on the host-mapped block when single-rank and untimed, else a copy)
static int collect_scalars(vlgba_ctx *c, bool spin, double hs[6])
{
    ba_dev &d = c->d;
    // new SSE, camera and point parts of dp'(lambda dp + g), and the solve's
    // two status words (every rank then takes the same pinv / re-solve
    // decision; scal[0] = the global old SSE, schur_phase)
    if (c->world > 1 || c->comm) TRY(allreduce(c, d.scal + 1, 5));
    if (spin) {
        // spin on the host-mapped sequence number written last (by the update's
        // final sums, or k_publish); lower latency than a copy +
        // hipStreamSynchronize.  A stalled stream falls back to the
        // synchronisation, which reports the error
        if (!d.published) TRY(ba_launch_publish(&d));
        const double want = (double)d.seq;
        const auto t0 = std::chrono::steady_clock::now();
        bool got = false;
        for (long it = 0;; it++) {
            if (d.hres[7] == want) {
                got = true;
                break;
            }
            if ((it & 1023) == 1023 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
                break;
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (got) {
            for (int q = 0; q < 6; q++) hs[q] = d.hres[q];
            return 0;
        }
        VLGBA_CHECK(hipStreamSynchronize(d.stream));
    }
    TRY(download(hs, d.scal, 6, d.stream));
    VLGBA_CHECK(hipStreamSynchronize(d.stream));
    return 0;
}

// A hand-off spin of the one-launch solve gave up (timeout word scal[5]):
// nothing is wrong with S, the launch just did not finish in time.  Re-form
// S and e_ (the solve works in place), solve with the launches that never
// wait on other workgroups, then the same update.  Every rank gets here
// together (the status words travel in the scalars' all-reduce), so the
// collectives of schur_phase pair up.
static int resolve_nospin(vlgba_ctx *c, double lam, double hs[6])
{
    ba_dev &d = c->d;
    TRY(schur_phase(c, lam));
    TRY(ba_launch_assemble(&d));
    TRY(ba_chol_solve(&d, 1));
    d.publish_req = 0;
    d.published = 0;
    TRY(ba_launch_update(&d, lam, c->flags));
    if (d.parity) TRY(ba_launch_parity_new_sums(&d, lam));
    TRY(collect_scalars(c, false, hs));
    c->spin_retries++;
    // one of the envelope runner's own hand-offs gave up (most likely its side
    // stream sharing a hardware queue with the library stream, so the column
    // launches queue behind it): this context's column launches alone from now on
    TRY(std::min(0, ba_env_runner_timed_out(&d)));
    return 0;
}

// rocSOLVER's symmetric eigensolver, loaded on first use (the library is
// ~0.9 GB; a pass that never meets a non-positive pivot never loads it)
namespace {
struct rs_api {
    rocblas_status (*create)(rocblas_handle *);
    rocblas_status (*set_stream)(rocblas_handle, hipStream_t);
    rocblas_status (*syevd)(rocblas_handle, const rocblas_evect, const rocblas_fill,
                            const rocblas_int, double *, const rocblas_int, double *, double *,
                            rocblas_int *);
    rocblas_status (*potrf)(rocblas_handle, const rocblas_fill, const rocblas_int, double *,
                            const rocblas_int, rocblas_int *);
    rocblas_status (*potrs)(rocblas_handle, const rocblas_fill, const rocblas_int,
                            const rocblas_int, double *, const rocblas_int, double *,
                            const rocblas_int);
    bool ok = false;
};
rs_api *rs_load()
{
    static rs_api api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        api.create = (decltype(api.create))dlsym(h, "rocblas_create_handle");
        api.set_stream = (decltype(api.set_stream))dlsym(h, "rocblas_set_stream");
        api.syevd = (decltype(api.syevd))dlsym(h, "rocsolver_dsyevd");
        api.potrf = (decltype(api.potrf))dlsym(h, "rocsolver_dpotrf");
        api.potrs = (decltype(api.potrs))dlsym(h, "rocsolver_dpotrs");
        api.ok = api.create && api.set_stream && api.syevd;
    });
    return api.ok ? &api : nullptr;
}
std::mutex g_rs_mu;
std::map<int, rocblas_handle> g_rs_handle;   // per device
}   // namespace

// da = pinv(S) * e_ on the GPU (bundle_euclid.m:193) for a pass whose
// Cholesky met a non-positive pivot: S and e_ again (the solve overwrote them
// in place), the lower triangle of S assembled densely, rocSOLVER dsyevd,
// then V diag(1/ev, |ev| > tol) V^T e_ (ba_pinv_apply), and the update with
// that da.  Every rank runs it on the identical all-reduced system.
// rocSOLVER, the dense scratch of the fallbacks and this device's handle
static int rs_prepare(vlgba_ctx *c, rs_api **rs_out, rocblas_handle *hdl_out)
{
    ba_dev &d = c->d;
    rs_api *rs = rs_load();
    if (!rs) return VLGBA_E_ARG;
    const long long ld = d.ld;
    if (ld > 0x7fffffffLL) return VLGBA_E_ARG;
    if (!c->pinv_S) {
        TRY(dalloc(&c->pinv_S, (size_t)(ld * ld)));
        TRY(dalloc(&c->pinv_ev, (size_t)ld));
        TRY(dalloc(&c->pinv_e, (size_t)ld));
        TRY(dalloc(&c->pinv_w, (size_t)ld));
        TRY(dalloc(&c->pinv_info, 1));
    }
    rocblas_handle hdl = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        auto it = g_rs_handle.find(d.device);
        if (it == g_rs_handle.end()) {
            if (rs->create(&hdl) != rocblas_status_success) return VLGBA_E_ARG;
            g_rs_handle[d.device] = hdl;
        } else {
            hdl = it->second;
        }
    }
    *rs_out = rs;
    *hdl_out = hdl;
    return 0;
}

// A pass whose nested-dissection Cholesky met a non-positive pivot: the same
// S (the Cholesky took it in place) is assembled densely in the natural
// camera order and factored by rocSOLVER dpotrf before the pinv fallback is
// considered -- the pivot may be an artefact of the elimination order on a
// system whose gauge directions only the damping lifts (cond(S) up to 1e17 on
// the growing replays), and the natural order is the one bundle_euclid.m's
// pinv is then compared with.  Returns 1 if dpotrf fails
// too (the caller takes the pinv step), 0 with the pass finished.
static int nd_natural_retry(vlgba_ctx *c, double lam, double hs[6])
{
    ba_dev &d = c->d;
    rs_api *rs = nullptr;
    rocblas_handle hdl = nullptr;
    TRY(rs_prepare(c, &rs, &hdl));
    if (!rs->potrf || !rs->potrs) return 1;
    const long long ld = d.ld;
    TRY(schur_phase(c, lam));
    TRY(ba_launch_assemble_plain(&d, c->pinv_S, ld, 1));
    TRY(ba_fix_diag_plain(&d, c->pinv_S, ld));   // exactly-zero rows: unit diagonal, rhs 0
    VLGBA_CHECK(hipMemcpyAsync(c->pinv_e, d.rhs, sizeof(double) * ld, hipMemcpyDeviceToDevice,
                               d.stream));
    VLGBA_CHECK(hipStreamSynchronize(d.stream));
    int info = 0;
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        if (rs->set_stream(hdl, d.stream) != rocblas_status_success ||
            rs->potrf(hdl, rocblas_fill_lower, (rocblas_int)ld, c->pinv_S, (rocblas_int)ld,
                      c->pinv_info) != rocblas_status_success)
            return VLGBA_E_ARG;
        VLGBA_CHECK(hipMemcpyAsync(&info, c->pinv_info, sizeof info, hipMemcpyDeviceToHost,
                                   d.stream));
        VLGBA_CHECK(hipStreamSynchronize(d.stream));
        if (info != 0) return 1;
        if (rs->potrs(hdl, rocblas_fill_lower, (rocblas_int)ld, 1, c->pinv_S, (rocblas_int)ld,
                      c->pinv_e, (rocblas_int)ld) != rocblas_status_success)
            return VLGBA_E_ARG;
    }
    VLGBA_CHECK(hipMemcpyAsync(d.da, c->pinv_e, sizeof(double) * ld, hipMemcpyDeviceToDevice,
                               d.stream));
    d.publish_req = 0;
    d.published = 0;
    TRY(ba_launch_update(&d, lam, c->flags));
    if (d.parity) TRY(ba_launch_parity_new_sums(&d, lam));
    TRY(collect_scalars(c, false, hs));
    c->nd_retries++;
    if (c->rank == 0 && !std::getenv("VLGBA_QUIET"))
        std::fprintf(stderr, "[vlgba] non-positive pivot in the nested-dissection order: the "
                             "natural-order Cholesky (dpotrf) took the pass\n");
    return 0;
}

static int pinv_fallback(vlgba_ctx *c, double lam, double hs[6])
{
    ba_dev &d = c->d;
    const auto t0 = std::chrono::steady_clock::now();
    rs_api *rs = nullptr;
    rocblas_handle hdl = nullptr;
    TRY(rs_prepare(c, &rs, &hdl));
    const long long ld = d.ld;
    TRY(schur_phase(c, lam));
    TRY(ba_launch_assemble_plain(&d, c->pinv_S, ld, 1));
    // the library stream is non-blocking: make S complete before rocSOLVER
    // (parts of dsyevd are ordered against the legacy stream, not ours)
    VLGBA_CHECK(hipStreamSynchronize(d.stream));
    {
        std::lock_guard<std::mutex> lk(g_rs_mu);
        if (rs->set_stream(hdl, d.stream) != rocblas_status_success ||
            rs->syevd(hdl, rocblas_evect_original, rocblas_fill_lower, (rocblas_int)ld,
                      c->pinv_S, (rocblas_int)ld, c->pinv_ev, c->pinv_e,
                      c->pinv_info) != rocblas_status_success)
            return VLGBA_E_ARG;
        VLGBA_CHECK(hipStreamSynchronize(d.stream));
    }
    {
        int info = 0;
        VLGBA_CHECK(hipMemcpy(&info, c->pinv_info, sizeof info, hipMemcpyDeviceToHost));
        if (info != 0) return VLGBA_E_ARG;   // the eigensolver did not converge
    }
    TRY(ba_pinv_apply(&d, c->pinv_S, c->pinv_ev, ld, d.rhs, c->pinv_w, d.da));
    d.publish_req = 0;
    d.published = 0;
    TRY(ba_launch_update(&d, lam, c->flags));
    if (d.parity) TRY(ba_launch_parity_new_sums(&d, lam));
    TRY(collect_scalars(c, false, hs));
    c->pinv_used++;
    if (c->rank == 0 && !std::getenv("VLGBA_QUIET"))
        std::fprintf(stderr,
                     "[vlgba] non-positive pivot: da = pinv(S) e_ by dsyevd on the dense "
                     "%lld x %lld S (%.1f MB of device memory), %.3f s\n",
                     ld, ld, 8e-6 * (double)ld * (double)ld,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return 0;
}

static int lm_pass(vlgba_ctx *c, int relinearize, vlgba_step_info *info)
{
    ba_dev &d = c->d;
    const double lam = c->lambda;
    mark(c, 0);
    // fused update: every pass's update linearises at the new point (into the
    // second buffers, swapped in on accept), so a pass linearises here only
    // after set_params; relinearize then means the camera reduction of the
    // current linearisation (the rest of stage 1), the work an accepted pass
    // does
    const bool full = !c->lin_valid || (relinearize && !d.fused);
    if (full || (d.fused && (relinearize || c->camred_due))) {
        // the rotation table of d.a is current: set_params builds it and an
        // accepted step swaps in the one k_camera_update built for a_new
        if (full) TRY(ba_launch_linearize(&d, c->flags));
        mark(c, 1);
        if (!d.ordered && d.fuse_camred && d.ngrp_mf > 0) {
            // U / eA / old SSE: workgroups of this pass's MFMA Schur launch
            TRY(ba_launch_camera_reduce(&d, c->flags, 1));
        } else if (!d.ordered && c->world == 1 && !c->timing) {
            // U / eA / old SSE on the side stream, overlapping V*^-1 and the
            // Schur chunks (no collective in between at world size 1);
            // launch_schur_fast joins before k_schur_reduce
            VLGBA_CHECK(hipEventRecord(d.ev_fork, d.stream));
            VLGBA_CHECK(hipStreamWaitEvent(d.side, d.ev_fork, 0));
            hipStream_t s0 = d.stream;
            d.stream = d.side;
            const int rc = ba_launch_camera_reduce(&d, c->flags);
            d.stream = s0;
            TRY(rc);
            VLGBA_CHECK(hipEventRecord(d.ev_join, d.side));
            d.join_pending = 1;
        } else {
            TRY(ba_launch_camera_reduce(&d, c->flags));
        }
        if (d.parity) TRY(ba_launch_parity_old_sse(&d));
        // U | eA | old_sse travel in one all-reduce (the fast path's reduce
        // kernel writes the old_sse slot itself)
        if (d.ordered)
            VLGBA_CHECK(hipMemcpyAsync(d.eA + d.ld, d.scal + 0, sizeof(double),
                                       hipMemcpyDeviceToDevice, d.stream));
        c->lin_valid = 1;
        c->camred_due = 0;
    } else {
        mark(c, 1);
    }
    TRY(schur_phase(c, lam));
    mark(c, 4);
    TRY(ba_launch_assemble(&d));
    mark(c, 5);
    TRY(ba_chol_solve(&d));
    for (int w = 4; w <= 5; w++) {   // test hooks: as if a pivot failed / a spin gave up
        int &k = w == 4 ? c->debug_pivots : c->debug_timeouts;
        if (k > 0) {
            static const double one = 1.0;
            VLGBA_CHECK(hipMemcpyAsync(d.scal + w, &one, sizeof one, hipMemcpyHostToDevice,
                                       d.stream));
            k--;
        }
    }
    mark(c, 6);
    // RCCL ranks spin as well: their collectives are stream-ordered, and the
    // publish then follows the scalars' all-reduce (collect_scalars)
    const bool spin = (c->world == 1 || c->comm) && !c->timing;
    d.publish_req = spin && !c->comm;   // the fast update's final-sums launch publishes
    d.published = 0;
    TRY(ba_launch_update(&d, lam, c->flags));
    d.publish_req = 0;
    if (d.parity) TRY(ba_launch_parity_new_sums(&d, lam));
    mark(c, 7);
    // scalars: [0] old_sse [1] new_sse [2] dpg cameras [3] dpg points
    // [4] non-positive pivot [5] hand-off spin timeout (summed over ranks)
    double hs[6];
    TRY(collect_scalars(c, spin, hs));
    info->pinv = 0;
    info->spin_retry = 0;
    info->nd_retry = 0;
    if (hs[5] != 0.0) {   // the solve did not finish: again, without spins
        TRY(resolve_nospin(c, lam, hs));
        info->spin_retry = 1;
    }
    if (hs[4] != 0.0 && d.nd_np > 0) {   // the nested-dissection order's pivot: the
        const int rc = nd_natural_retry(c, lam, hs);   // natural order first
        if (rc < 0) return rc;
        info->nd_retry = 1;
        if (rc == 0) hs[4] = 0.0;
    }
    if (hs[4] != 0.0) {
        // non-positive pivot: bundle_euclid.m:193 takes pinv(S)*e_ whatever S is
        // (App. A Q8), so does the fallback -- then the same update
        TRY(pinv_fallback(c, lam, hs));
        info->pinv = 1;
    }
    if (c->timing) {
        float ms;
        const int map[7][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6}, {6, 7}};
        for (int q = 0; q < 7; q++) {
            (void)hipEventElapsedTime(&ms, c->ev[map[q][0]], c->ev[map[q][1]]);
            c->phase_ms[q] = ms;
        }
        ba_ktimer *kt = d.kt;
        for (int q = 0; kt && q + 1 < kt->nev; q += 2) {
            (void)hipEventElapsedTime(&ms, kt->ev[q], kt->ev[q + 1]);
            kt->ms[kt->kid[q / 2]] += ms;
            kt->calls[kt->kid[q / 2]]++;
        }
        if (kt) {
            kt->nev = 0;
            // the solve's algorithmic flops (ba_chol_setup's count) on the timers
            // that ran them: one-launch / per-level CR, or the envelope's steps,
            // separator SYRK and backward solve
            const bool cr = d.cr_nlev > 0;
            kt->flops[cr ? KT_CR_FACTOR : KT_FACTOR] += d.fl_factor;
            kt->flops[KT_SYRK] += d.fl_syrk;
            kt->flops[cr ? KT_CR_BACK : KT_BACKWARD] += d.fl_back;
        }
    }
    info->old_sse = hs[0];
    info->new_sse = hs[1];
    info->dpg = hs[2] + hs[3];
    info->lambda = lam;
    info->chol_failed = info->pinv;   // the Cholesky failed; the step is pinv(S)*e_
    info->rho = (hs[0] - hs[1]) / info->dpg;
    if (c->model == VLGBA_MODEL_PROJECTIVE)   // bundle_projective.m:182-188 (normalised first)
        info->accepted = 1 / c->num_vis * hs[1] < 1 / c->num_vis * hs[0];
    else                                      // bundle_euclid.m:218
        info->accepted = (hs[0] - hs[1]) > 0;
    return 0;
}

// bundle_euclid.m:218-241 (bundle_projective.m:188-207) applied to the context
static void lm_apply(vlgba_ctx *c, const vlgba_step_info *info)
{
    ba_dev &d = c->d;
    const bool proj = c->model == VLGBA_MODEL_PROJECTIVE;
    if (info->accepted) {
        std::swap(d.a, d.a_new);
        std::swap(d.b, d.b_new);
        std::swap(d.rot, d.rot_new);   // rotation table of the new a
        if (d.fused) {   // the update linearised at the new point: take it
            std::swap(d.W, d.W2);
            std::swap(d.V, d.V2);
            std::swap(d.eB, d.eB2);
            std::swap(d.upart, d.upart2);
            std::swap(d.chsse, d.chsse2);
        }
        if (proj)
            c->lambda = c->lambda / 10;
        else
            c->lambda = c->lambda * std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * info->rho - 1.0, 3));
        c->nu = 2.0;
        c->lin_valid = d.fused ? 1 : 0;
        c->camred_due = d.fused ? 1 : 0;
    } else if (proj) {
        c->lambda = c->lambda * 10;
    } else {
        c->lambda = c->lambda * c->nu;
        c->nu = 2.0 * c->nu;
    }
}

// every handle entry point runs on the context's device, whatever the calling
// thread's current device is (allocations and launches follow hipGetDevice)
static int ctx_enter(vlgba_ctx *c)
{
    return hipSetDevice(c->aux.device) == hipSuccess ? 0 : VLGBA_E_ARG;
}

// =========================================================================
// C ABI
// =========================================================================
extern "C" {

int vlgba_version(char *buf, int len)
{
    const int n = (int)std::strlen(VLGBA_VERSION_STR);
    if (buf && len > 0) {
        std::strncpy(buf, VLGBA_VERSION_STR, (size_t)len - 1);
        buf[len - 1] = 0;
    }
    return n;
}

int vlgba_abi_check(int abi_version, long long sz_problem, long long sz_options,
                    long long sz_stats, long long sz_step_info, long long sz_resect_problem)
{
    const bool ok = abi_version == VLGBA_ABI_VERSION &&
                    sz_problem == (long long)sizeof(vlgba_problem) &&
                    sz_options == (long long)sizeof(vlgba_options) &&
                    sz_stats == (long long)sizeof(vlgba_stats) &&
                    sz_step_info == (long long)sizeof(vlgba_step_info) &&
                    sz_resect_problem == (long long)sizeof(vlgba_resect_problem);
    return ok ? 0 : VLGBA_E_ABI;
}

int vlgba_get_unique_id(void *id128)
{
    if (!id128) return VLGBA_E_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return VLGBA_E_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id128, &id, sizeof id);
    return 0;
}

// the caller forgets a unique id: destroy the idle communicators made from it
// (contexts still holding one keep it until vlgba_destroy, which then
// destroys it as an unkeyed communicator).  Returns the number destroyed.
int vlgba_comm_release(const void *id128)
{
    if (!id128) return VLGBA_E_ARG;
    const std::string id((const char *)id128, 128);
    std::vector<ncclComm_t> drop;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        for (auto q = g_comm_idle.begin(); q != g_comm_idle.end();) {
            if (q->first.id == id) {
                drop.push_back(q->second);
                g_comm_key.erase(q->second);
                q = g_comm_idle.erase(q);
            } else {
                ++q;
            }
        }
        for (auto q = g_comm_key.begin(); q != g_comm_key.end();)   // in use: unkeyed,
            q = q->second.id == id ? g_comm_key.erase(q) : std::next(q);   // destroyed on release
    }
    for (ncclComm_t x : drop) ncclCommDestroy(x);
    return (int)drop.size();
}

int vlgba_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int vlgba_create(const vlgba_problem *prob, const vlgba_options *opt, vlgba_ctx **out)
{
    if (!out) return VLGBA_E_ARG;
    return ctx_create(prob, opt, out, true, true, false);
}

void vlgba_destroy(vlgba_ctx *ctx)
{
    if (ctx) (void)ctx_enter(ctx);
    ctx_free(ctx);
}

// per-point device array (k doubles per local point, internal order) -> host,
// in the input point order (synchronous when a permutation applies)
static int download_points(vlgba_ctx *c, double *dst, const double *src, int k)
{
    const size_t cnt = (size_t)k * c->d.n;
    if (c->pperm.empty()) return download(dst, src, cnt, c->d.stream);
    std::vector<double> tmp(cnt);
    TRY(download(tmp.data(), src, cnt, c->d.stream));
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    for (int i = 0; i < c->d.n; i++)
        std::memcpy(dst + (size_t)k * c->pperm[i], tmp.data() + (size_t)k * i, sizeof(double) * k);
    return 0;
}

int vlgba_set_params(vlgba_ctx *c, const double *a, const double *b)
{
    if (!c || !a || !b) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    static const bool pageable = std::getenv("VLGBA_SETP_PAGEABLE") != nullptr;   // A/B
    const size_t na = (size_t)c->d.ld, nb = 3 * (size_t)c->d.n;
    ba_aux &x = c->aux;
    if (!pageable && x.pin_cap < na + nb) {   // pinned staging: the copies start at once
        if (x.pin) (void)hipHostFree(x.pin);
        size_t cap = 1 << 16;
        while (cap < na + nb) cap <<= 1;
        x.pin = nullptr;
        x.pin_cap = 0;
        if (hipHostMalloc((void **)&x.pin, sizeof(double) * cap, hipHostMallocDefault) ==
            hipSuccess)
            x.pin_cap = cap;
    }
    double *ha = (!pageable && x.pin) ? x.pin : nullptr, *hb = ha ? ha + na : nullptr;
    if (ha) std::memcpy(ha, a, sizeof(double) * na);
    TRY(upload(c->d.a, ha ? ha : a, na, c->d.stream));
    if (!c->pperm.empty()) {   // input point order -> internal order
        double *dst = hb;
        if (!dst) {
            c->hb_tmp.resize(nb);
            dst = c->hb_tmp.data();
        }
        for (int i = 0; i < c->d.n; i++)
            for (int r = 0; r < 3; r++)
                dst[3 * (size_t)i + r] = b[3 * ((size_t)c->p0 + c->pperm[i]) + r];
        TRY(upload(c->d.b, dst, nb, c->d.stream));
    } else if (hb) {
        std::memcpy(hb, b + 3 * (size_t)c->p0, sizeof(double) * nb);
        TRY(upload(c->d.b, hb, nb, c->d.stream));
    } else {
        TRY(upload(c->d.b, b + 3 * (size_t)c->p0, nb, c->d.stream));
    }
    TRY(ba_launch_rotations(&c->d, c->d.a, c->d.rot, 1));
    c->lin_valid = 0;
    static const bool tm = std::getenv("VLGBA_SETP_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    if (tm)
        std::fprintf(stderr, "[vlgba set_params] m=%d sync %.3f ms\n", c->d.m,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                         .count());
    return 0;
}

int vlgba_get_params(vlgba_ctx *c, double *a, double *b)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    if (a) TRY(download(a, c->d.a, (size_t)c->d.ld, c->d.stream));
    if (b) {
        if (c->world > 1) {
            // every rank returns the full b: all-reduce of a zero-padded copy
            double *full = nullptr;
            TRY(dalloc(&full, 3 * (size_t)c->n_global));
            VLGBA_CHECK(hipMemsetAsync(full, 0, sizeof(double) * 3 * c->n_global, c->d.stream));
            if (c->pperm.empty()) {
                VLGBA_CHECK(hipMemcpyAsync(full + 3 * (size_t)c->p0, c->d.b,
                                           sizeof(double) * 3 * c->d.n, hipMemcpyDeviceToDevice,
                                           c->d.stream));
            } else {   // internal -> input order inside this rank's range
                c->hb_tmp.resize(3 * (size_t)c->d.n);
                TRY(download_points(c, c->hb_tmp.data(), c->d.b, 3));
                VLGBA_CHECK(hipMemcpyAsync(full + 3 * (size_t)c->p0, c->hb_tmp.data(),
                                           sizeof(double) * 3 * c->d.n, hipMemcpyHostToDevice,
                                           c->d.stream));
                VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
            }
            int rc = allreduce(c, full, 3 * (size_t)c->n_global);
            if (!rc) rc = download(b, full, 3 * (size_t)c->n_global, c->d.stream);
            (void)hipStreamSynchronize(c->d.stream);
            ba_dfree(full);
            if (rc) return rc;
        } else {
            TRY(download_points(c, b, c->d.b, 3));
        }
    }
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    return 0;
}

int vlgba_get_linearization(vlgba_ctx *c, double *U, double *eA, double *V, double *eB,
                            double *W)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    ba_dev &d = c->d;
    // the linearisation the context holds for the current parameters (a
    // rejected step's, or the one the fused update made at an accepted step's
    // new point), else a new one
    if (!c->lin_valid) {
        TRY(ba_launch_rotations(&d, d.a, d.rot, 1));
        TRY(ba_launch_linearize(&d, c->flags));
    }
    if (!c->lin_valid || c->camred_due) {
        TRY(ba_launch_camera_reduce(&d, c->flags));
        if (d.ordered)
            VLGBA_CHECK(hipMemcpyAsync(d.eA + d.ld, d.scal + 0, sizeof(double),
                                       hipMemcpyDeviceToDevice, d.stream));
    }
    c->lin_valid = 1;
    c->camred_due = 0;
    // U / eA stay per-rank partials on the device (schur_owner); the caller
    // gets their sum over ranks
    const size_t nue = (size_t)d.na * d.na * d.m + d.ld + 1;
    double *ue = d.U;
    if (c->world > 1) {
        TRY(dalloc(&ue, nue));
        VLGBA_CHECK(hipMemcpyAsync(ue, d.U, sizeof(double) * nue, hipMemcpyDeviceToDevice,
                                   d.stream));
        const int rc = allreduce(c, ue, nue);
        if (rc) {
            ba_dfree(ue);
            return rc;
        }
    }
    int rc = 0;
    if (U) rc = download(U, ue, (size_t)d.na * d.na * d.m, d.stream);
    if (!rc && eA) rc = download(eA, ue + (size_t)d.na * d.na * d.m, (size_t)d.ld, d.stream);
    if (ue != d.U) {
        (void)hipStreamSynchronize(d.stream);
        ba_dfree(ue);
    }
    TRY(rc);
    if (V) TRY(download_points(c, V, d.V, 9));
    if (eB) TRY(download_points(c, eB, d.eB, 3));
    if (W) {
        if (c->operm.empty()) {
            TRY(download(W, d.W, (size_t)3 * d.na * d.N, d.stream));
        } else {   // internal observation order -> input order
            const size_t ws = (size_t)3 * d.na;
            std::vector<double> tmp(ws * d.N);
            TRY(download(tmp.data(), d.W, ws * d.N, d.stream));
            VLGBA_CHECK(hipStreamSynchronize(d.stream));
            for (int o = 0; o < d.N; o++)
                std::memcpy(W + ws * c->operm[o], tmp.data() + ws * o, sizeof(double) * ws);
        }
    }
    VLGBA_CHECK(hipStreamSynchronize(d.stream));
    return 0;
}

int vlgba_get_reduced_system(vlgba_ctx *c, int *blk_jk, double *blocks, double *e_)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    ba_dev &d = c->d;
    if (!c->lin_valid || c->camred_due) {   // stage 1 at the current parameters (as a
        if (!c->lin_valid) TRY(ba_launch_linearize(&d, c->flags));   // pass would)
        TRY(ba_launch_camera_reduce(&d, c->flags));
        c->camred_due = 0;
        if (d.ordered)
            VLGBA_CHECK(hipMemcpyAsync(d.eA + d.ld, d.scal + 0, sizeof(double),
                                       hipMemcpyDeviceToDevice, d.stream));
        c->lin_valid = 1;
    }
    TRY(schur_phase(c, c->lambda));
    if (d.join_pending) {
        VLGBA_CHECK(hipStreamWaitEvent(d.stream, d.ev_join, 0));
        d.join_pending = 0;
    }
    if (blk_jk) TRY(download(blk_jk, d.blk_jk, 2 * (size_t)d.nb, d.stream));
    if (blocks) TRY(download(blocks, d.sblk, (size_t)d.na * d.na * d.nb, d.stream));
    if (e_) TRY(download(e_, d.rhs, (size_t)d.ld, d.stream));
    VLGBA_CHECK(hipStreamSynchronize(d.stream));
    return 0;
}

int vlgba_get_step(vlgba_ctx *c, double *da, double *db)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    if (da) TRY(download(da, c->d.da, (size_t)c->d.ld, c->d.stream));
    if (db) TRY(download_points(c, db, c->d.db, 3));
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    return 0;
}

int vlgba_debug_force_status(vlgba_ctx *c, int word, int passes)
{
    if (!c || word < 4 || word > 6 || passes < 0) return VLGBA_E_ARG;
    if (word == 6)
        c->d.debug_runner_fail = passes;
    else
        (word == 4 ? c->debug_pivots : c->debug_timeouts) = passes;
    return 0;
}

int vlgba_set_timing(vlgba_ctx *c, int on)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    if (on && !c->ev[0])
        for (auto &e : c->ev) VLGBA_CHECK(hipEventCreate(&e));
    if (on && !c->d.kt) {
        c->d.kt = new (std::nothrow) ba_ktimer();
        if (!c->d.kt) return VLGBA_E_NOMEM;
    }
    c->timing = on;
    if (c->d.kt) c->d.kt->on = on;
    return 0;
}

// kernel times of the contexts destroyed with timing on (VLGBA_KTIME_ALL=1:
// every context times its passes -- the growing replay's device-busy split)
static std::mutex g_kt_mu;
static double g_kt_ms[KT_N], g_kt_flops[KT_N];
static long long g_kt_calls[KT_N];

static void kt_retire(const ba_ktimer *kt)
{
    std::lock_guard<std::mutex> lk(g_kt_mu);
    for (int k = 0; k < KT_N; k++) {
        g_kt_ms[k] += kt->ms[k];
        g_kt_calls[k] += kt->calls[k];
        g_kt_flops[k] += kt->flops[k];
    }
}

int vlgba_kernel_ms(vlgba_ctx *c, double *ms, long long *calls, int reset)
{
    if (!c) {   // process-wide: the destroyed contexts' timers
        std::lock_guard<std::mutex> lk(g_kt_mu);
        for (int k = 0; k < KT_N; k++) {
            if (ms) ms[k] = g_kt_ms[k];
            if (calls) calls[k] = g_kt_calls[k];
            if (reset) {
                g_kt_ms[k] = 0.0;
                g_kt_calls[k] = 0;
                g_kt_flops[k] = 0.0;
            }
        }
        return 0;
    }
    if (!c->d.kt) return VLGBA_E_ARG;
    for (int k = 0; k < KT_N; k++) {
        if (ms) ms[k] = c->d.kt->ms[k];
        if (calls) calls[k] = c->d.kt->calls[k];
        if (reset) {
            c->d.kt->ms[k] = 0.0;
            c->d.kt->calls[k] = 0;
            c->d.kt->flops[k] = 0.0;
        }
    }
    return 0;
}

int vlgba_kernel_flops(vlgba_ctx *c, double *flops)
{
    if (!flops) return VLGBA_E_ARG;
    if (!c) {
        std::lock_guard<std::mutex> lk(g_kt_mu);
        for (int k = 0; k < KT_N; k++) flops[k] = g_kt_flops[k];
        return 0;
    }
    if (!c->d.kt) return VLGBA_E_ARG;
    for (int k = 0; k < KT_N; k++) flops[k] = c->d.kt->flops[k];
    return 0;
}

const char *vlgba_kernel_name(int k)
{
    static const char *names[KT_N] = {
        "k_rotations", "k_linearize", "k_camera_reduce", "k_damp_point", "k_schur",
        "k_schur_group", "k_schur_reduce", "k_assemble", "k_factor_step", "k_syrk",
        "k_backward", "k_camera_update", "k_point_update", "k_cr_factor", "k_cr_update",
        "k_cr_back", "k_schur_mfma", "k_update_linearize"};
    return (k >= 0 && k < KT_N) ? names[k] : "";
}

int vlgba_plan_info(vlgba_ctx *c, long long *info, int len)
{
    if (!c || !info) return VLGBA_E_ARG;
    const ba_dev &d = c->d;
    const long long ne = d.cr_nlev ? d.cr_eptr_h[d.cr_nlev] : 0;
    const long long nk = d.cr_nlev ? d.cr_kptr_h[d.cr_nlev] : 0;
    const long long v[VLGBA_NPLAN] = {d.N,   d.n,    d.m,   d.na,         d.nch,  d.ns,
                                      d.nes, d.ngrp, d.ngs, d.nge,        d.nb,   d.nt,
                                      d.cr_nlev, ne, nk,    d.ordered,    d.ordered ? d.T : d.nterm_fast,
                                      d.blob_words, d.mfma,
                                      d.cr_nlev ? (d.cr32 ? d.tb32 : 64) : 0,
                                      d.ngrp_mf, c->pperm.empty() ? 0 : 1, d.nl, d.nd_np,
                                      d.nd_np ? d.nt - d.nd_a0[d.nd_np] : 0,
                                      (long long)d.fl_factor, (long long)d.fl_syrk,
                                      (long long)d.fl_back, d.runner_runs};
    for (int k = 0; k < len && k < VLGBA_NPLAN; k++) info[k] = v[k];
    return VLGBA_NPLAN;
}

int vlgba_phase_ms(vlgba_ctx *c, double *ms7)
{
    if (!c || !ms7) return VLGBA_E_ARG;
    for (int q = 0; q < 7; q++) ms7[q] = c->phase_ms[q];
    return 0;
}

int vlgba_sync(vlgba_ctx *c)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    return 0;
}

int vlgba_step(vlgba_ctx *c, int relinearize, int update_lm, vlgba_step_info *info)
{
    if (!c) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    vlgba_step_info tmp;
    if (!info) info = &tmp;
    TRY(lm_pass(c, relinearize, info));
    if (update_lm) lm_apply(c, info);
    return 0;
}

int vlgba_run_passes(vlgba_ctx *c, int npass, vlgba_step_info *info)
{
    if (!c || npass < 0) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    vlgba_step_info tmp;
    if (!info) info = &tmp;
    std::memset(info, 0, sizeof *info);
    for (int q = 0; q < npass; q++) TRY(lm_pass(c, 1, info));
    return 0;
}

// bundle_euclid.m:111-249
int vlgba_run(vlgba_ctx *c, double *error_out, int error_cap, vlgba_stats *stats)
{
    if (!c || (error_out && error_cap < 0)) return VLGBA_E_ARG;
    TRY(ctx_enter(c));
    auto t0 = std::chrono::steady_clock::now();
    c->lambda = c->lambda0;
    c->nu = 2.0;
    c->lin_valid = 0;
    std::vector<double> err;   // error_, 1-based in the reference
    int iter = 1, iter2 = 0, passes = 0, acc = 0;
    const int pinv0 = c->pinv_used, retry0 = c->spin_retries, nd0 = c->nd_retries;
    for (;;) {
        if (!(iter < c->max_iter && iter2 < c->max_iter2)) break;
        if (iter >= 3) {
            const double e1 = err[iter - 1], e0 = err[iter - 2];
            if (!(e1 > 1e-20 && e0 - e1 > c->stop_rel * e0)) break;
        }
        vlgba_step_info info;
        TRY(lm_pass(c, 0, &info));
        passes++;
        if (info.accepted) {
            const bool proj = c->model == VLGBA_MODEL_PROJECTIVE;
            // bundle_euclid.m:219-220 divide; bundle_projective.m:182-183 scale by 1/num_vis
            const double olde = proj ? 1 / c->num_vis * info.old_sse : info.old_sse / c->num_vis;
            const double newe = proj ? 1 / c->num_vis * info.new_sse : info.new_sse / c->num_vis;
            if (c->verbose && c->rank == 0)
                std::printf("iter %d: error= %.5g -> %.5g\n", iter, olde, newe);
            if ((int)err.size() < iter) err.push_back(olde);
            else err[iter - 1] = olde;
            iter++;
            err.push_back(newe);
            iter2 = 0;
            acc++;
        } else {
            iter2++;
        }
        lm_apply(c, &info);
        if (c->on_pass && c->rank == 0) c->on_pass(passes, iter, &info, c->on_pass_user);
    }
    VLGBA_CHECK(hipStreamSynchronize(c->d.stream));
    if (error_out)   // at most error_cap entries; stats->num_error is the full count
        for (size_t q = 0; q < err.size() && q < (size_t)error_cap; q++) error_out[q] = err[q];
    if (stats) {
        stats->iterations = passes;
        stats->accepted = acc;
        stats->num_error = (int)err.size();
        stats->lambda = c->lambda;
        stats->pinv_passes = c->pinv_used - pinv0;
        stats->spin_retries = c->spin_retries - retry0;
        stats->nd_retries = c->nd_retries - nd0;
        stats->seconds =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return 0;
}

int vlgba_solve(const vlgba_problem *prob, const vlgba_options *opt, double *a, double *b,
                double *error_out, int error_cap, vlgba_stats *stats)
{
    if (!a || !b) return VLGBA_E_ARG;
    vlgba_ctx *c = nullptr;
    TRY(vlgba_create(prob, opt, &c));
    int rc = vlgba_set_params(c, a, b);
    if (!rc) rc = vlgba_run(c, error_out, error_cap, stats);
    if (!rc) rc = vlgba_get_params(c, a, b);
    vlgba_destroy(c);
    return rc;
}

// ---------------------------------------------------------------------------
// stage entries (MEX layouts)
// ---------------------------------------------------------------------------
static void obs_from_vis(int m, int n, const double *vis, std::vector<int> &pt,
                         std::vector<int> &cam)
{
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++)
            if (vis[i + (size_t)n * j] != 0.0) {
                pt.push_back(i);
                cam.push_back(j);
            }
}

static int mex1_impl(int model, int m, int n, int num_a, const double *K, const double *a,
                     const double *b, const double *X, const double *vis, double *X_hat,
                     double *A, double *B, double *e, double *U, double *V, double *W,
                     double *eA, double *eB)
{
    if (m < 1 || n < 0 || (!K && model == VLGBA_MODEL_EUCLIDEAN) || !a || !b || !X || !vis)
        return VLGBA_E_ARG;
    std::vector<int> pt, cam;
    obs_from_vis(m, n, vis, pt, cam);
    const long long N = (long long)pt.size();
    std::vector<double> ox(2 * N);
    for (long long q = 0; q < N; q++) {
        const size_t p = (size_t)pt[q] + (size_t)n * cam[q];
        ox[2 * q] = X[2 * p];
        ox[2 * q + 1] = X[2 * p + 1];
    }
    vlgba_problem pr = {m, n, num_a, N, pt.data(), cam.data(), ox.data(), K, 0.0, model};
    vlgba_ctx *c = nullptr;
    TRY(ctx_create(&pr, nullptr, &c, true, true, true));
    ba_dev &d = c->d;
    int rc = 0;
    std::vector<double> jr((size_t)d.js * N), hW((size_t)3 * num_a * N), xh(2 * N), hB(6 * N);
    do {
        if ((rc = ctx_alloc(c, &d.xh_out, 2 * (size_t)N))) break;
        if ((rc = ctx_alloc(c, &d.B_out, 6 * (size_t)N))) break;
        if ((rc = upload(d.a, a, (size_t)d.ld, d.stream))) break;
        if ((rc = upload(d.b, b, 3 * (size_t)n, d.stream))) break;
        ba_flags f = {0, 0, 0};
        if ((rc = ba_launch_rotations(&d, d.a, d.rot, 1))) break;
        if ((rc = ba_launch_linearize(&d, f))) break;
        if ((rc = ba_launch_camera_reduce(&d, f))) break;
        if ((rc = download(jr.data(), d.jrec, jr.size(), d.stream))) break;
        if ((rc = download(hW.data(), d.W, hW.size(), d.stream))) break;
        if ((rc = download(xh.data(), d.xh_out, xh.size(), d.stream))) break;
        if ((rc = download(hB.data(), d.B_out, hB.size(), d.stream))) break;
        if ((rc = download(U, d.U, (size_t)num_a * num_a * m, d.stream))) break;
        if ((rc = download(eA, d.eA, (size_t)num_a * m, d.stream))) break;
        if ((rc = download(V, d.V, 9 * (size_t)n, d.stream))) break;
        if ((rc = download(eB, d.eB, 3 * (size_t)n, d.stream))) break;
        if (hipStreamSynchronize(d.stream) != hipSuccess) { rc = -1; break; }
    } while (0);
    ctx_free(c);
    if (rc) return rc;
    // scatter to the dense MEX layouts; invisible pairs: X_hat = X, zeros
    const size_t nm = (size_t)n * m;
    for (size_t p = 0; p < nm; p++) {
        X_hat[2 * p] = X[2 * p];
        X_hat[2 * p + 1] = X[2 * p + 1];
        e[2 * p] = e[2 * p + 1] = 0.0;
    }
    std::memset(A, 0, sizeof(double) * 2 * num_a * nm);
    std::memset(B, 0, sizeof(double) * 6 * nm);
    std::memset(W, 0, sizeof(double) * 3 * num_a * nm);
    const int js = 2 * num_a + 2;
    for (long long q = 0; q < N; q++) {
        const size_t p = (size_t)pt[q] + (size_t)n * cam[q];
        X_hat[2 * p] = xh[2 * q];
        X_hat[2 * p + 1] = xh[2 * q + 1];
        std::memcpy(A + 2 * num_a * p, jr.data() + js * q, sizeof(double) * 2 * num_a);
        e[2 * p] = jr[js * q + 2 * num_a];
        e[2 * p + 1] = jr[js * q + 2 * num_a + 1];
        std::memcpy(B + 6 * p, hB.data() + 6 * q, sizeof(double) * 6);
        std::memcpy(W + 3 * num_a * p, hW.data() + 3 * num_a * q, sizeof(double) * 3 * num_a);
    }
    return 0;
}

static int mex2_impl(int model, int m, int n, int num_a, const double *Y, const double *W,
                     const double *U, const double *eA, const double *eB, double *S,
                     double *e_)
{
    if (m < 1 || n < 0 || !Y || !W || !U || !eA || !eB || !S || !e_) return VLGBA_E_ARG;
    const int bs = 3 * num_a;
    std::vector<int> pt, cam;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) {
            const size_t p = (size_t)i + (size_t)n * j;
            bool nz = false;
            for (int q = 0; q < bs && !nz; q++) nz = (Y[bs * p + q] != 0.0) || (W[bs * p + q] != 0.0);
            if (nz) {
                pt.push_back(i);
                cam.push_back(j);
            }
        }
    const long long N = (long long)pt.size();
    std::vector<double> ox(2 * N, 0.0), hY((size_t)bs * N), hW((size_t)bs * N);
    for (long long q = 0; q < N; q++) {
        const size_t p = (size_t)pt[q] + (size_t)n * cam[q];
        std::memcpy(hY.data() + bs * q, Y + bs * p, sizeof(double) * bs);
        std::memcpy(hW.data() + bs * q, W + bs * p, sizeof(double) * bs);
    }
    std::vector<double> K(4 * (size_t)m, 1.0);
    vlgba_problem pr = {m, n, num_a, N, pt.data(), cam.data(), ox.data(), K.data(), 0.0, model};
    vlgba_ctx *c = nullptr;
    TRY(ctx_create(&pr, nullptr, &c, false, true, true));
    ba_dev &d = c->d;
    const long long ld = d.ld;
    int rc = 0;
    double *Sd = nullptr;
    do {
        if ((rc = ctx_alloc(c, &Sd, (size_t)(ld * ld)))) break;
        if ((rc = upload(d.Y, hY.data(), hY.size(), d.stream))) break;
        if ((rc = upload(d.W, hW.data(), hW.size(), d.stream))) break;
        if ((rc = upload(d.U, U, (size_t)num_a * num_a * m, d.stream))) break;
        if ((rc = upload(d.eA, eA, (size_t)num_a * m, d.stream))) break;
        if ((rc = upload(d.eB, eB, 3 * (size_t)n, d.stream))) break;
        if ((rc = ba_launch_yeb(&d))) break;
        // U is given already damped (bundle_euclid.m:192 passes U_): lambda = 0
        if ((rc = ba_launch_schur(&d, 0.0))) break;
        if ((rc = ba_launch_assemble_plain(&d, Sd, ld, 0))) break;
        if ((rc = download(S, Sd, (size_t)(ld * ld), d.stream))) break;
        if ((rc = download(e_, d.rhs, (size_t)ld, d.stream))) break;
        if (hipStreamSynchronize(d.stream) != hipSuccess) { rc = -1; break; }
    } while (0);
    ctx_free(c);
    return rc;
}

static int mex3_impl(int model, int m, int n, int num_a, const double *W, const double *da,
                     const double *eB, const double *Vinv, const double *K, const double *a,
                     const double *b, const double *X, const double *vis, double *db,
                     double *a_new, double *b_new, double *X_hat)
{
    if (m < 1 || n < 0 || !W || !da || !eB || !Vinv ||
        (!K && model == VLGBA_MODEL_EUCLIDEAN) || !a || !b || !X || !vis)
        return VLGBA_E_ARG;
    const int bs = 3 * num_a;
    std::vector<int> pt, cam;
    std::vector<unsigned char> ov;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) {
            const size_t p = (size_t)i + (size_t)n * j;
            bool nz = vis[p] != 0.0;
            const bool v = nz;
            for (int q = 0; q < bs && !nz; q++) nz = W[bs * p + q] != 0.0;
            if (nz) {
                pt.push_back(i);
                cam.push_back(j);
                ov.push_back(v ? 1 : 0);
            }
        }
    const long long N = (long long)pt.size();
    std::vector<double> ox(2 * N), hW((size_t)bs * N), xh(2 * N);
    for (long long q = 0; q < N; q++) {
        const size_t p = (size_t)pt[q] + (size_t)n * cam[q];
        ox[2 * q] = X[2 * p];
        ox[2 * q + 1] = X[2 * p + 1];
        std::memcpy(hW.data() + bs * q, W + bs * p, sizeof(double) * bs);
    }
    vlgba_problem pr = {m, n, num_a, N, pt.data(), cam.data(), ox.data(), K, 0.0, model};
    vlgba_ctx *c = nullptr;
    TRY(ctx_create(&pr, nullptr, &c, true, true, true));
    ba_dev &d = c->d;
    int rc = 0;
    do {
        if ((rc = ctx_alloc(c, &d.xh_out, 2 * (size_t)N))) break;
        if ((rc = ctx_alloc(c, &d.obs_vis, (size_t)N))) break;
        if ((rc = upload(d.obs_vis, ov.data(), ov.size(), d.stream))) break;
        if ((rc = upload(d.W, hW.data(), hW.size(), d.stream))) break;
        if ((rc = upload(d.da, da, (size_t)d.ld, d.stream))) break;
        if ((rc = upload(d.eB, eB, 3 * (size_t)n, d.stream))) break;
        if ((rc = upload(d.Vinv, Vinv, 9 * (size_t)n, d.stream))) break;
        if ((rc = upload(d.a, a, (size_t)d.ld, d.stream))) break;
        if ((rc = upload(d.b, b, 3 * (size_t)n, d.stream))) break;
        VLGBA_CHECK(hipMemsetAsync(d.eA, 0, sizeof(double) * d.ld, d.stream));
        if ((rc = ba_launch_update(&d, 0.0, ba_flags{}))) break;
        if ((rc = download(db, d.db, 3 * (size_t)n, d.stream))) break;
        if ((rc = download(a_new, d.a_new, (size_t)d.ld, d.stream))) break;
        if ((rc = download(b_new, d.b_new, 3 * (size_t)n, d.stream))) break;
        if ((rc = download(xh.data(), d.xh_out, xh.size(), d.stream))) break;
        if (hipStreamSynchronize(d.stream) != hipSuccess) { rc = -1; break; }
    } while (0);
    ctx_free(c);
    if (rc) return rc;
    const size_t nm = (size_t)n * m;
    for (size_t p = 0; p < nm; p++) {
        X_hat[2 * p] = X[2 * p];
        X_hat[2 * p + 1] = X[2 * p + 1];
    }
    for (long long q = 0; q < N; q++) {
        if (!ov[q]) continue;
        const size_t p = (size_t)pt[q] + (size_t)n * cam[q];
        X_hat[2 * p] = xh[2 * q];
        X_hat[2 * p + 1] = xh[2 * q + 1];
    }
    return 0;
}

int vlgba_debug_pinv_solve(int ld, const double *S, const double *e_, double *da)
{
    if (ld < 1 || !S || !e_ || !da) return VLGBA_E_ARG;
    rs_api *rs = rs_load();
    if (!rs) return VLGBA_E_ARG;
    int dev = 0;
    VLGBA_CHECK(hipGetDevice(&dev));
    ba_dev d;
    std::memset(&d, 0, sizeof d);
    d.device = dev;
    d.stream = nullptr;   // legacy stream: synchronous below
    double *buf = nullptr;
    int *info = nullptr;
    const size_t n = (size_t)ld;
    TRY(dalloc(&buf, n * n + 4 * n));
    int rc = dalloc(&info, 1);
    rocblas_handle hdl = nullptr;
    do {
        if (rc) break;
        double *A = buf, *ev = buf + n * n, *e = ev + n, *w = e + n, *rhs = w + n;
        if (hipMemcpy(A, S, sizeof(double) * n * n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(rhs, e_, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) {
            rc = -1;
            break;
        }
        if (rs->create(&hdl) != rocblas_status_success ||
            rs->syevd(hdl, rocblas_evect_original, rocblas_fill_lower, ld, A, ld, ev, e, info) !=
                rocblas_status_success) {
            rc = VLGBA_E_ARG;
            break;
        }
        if ((rc = ba_pinv_apply(&d, A, ev, ld, rhs, w, e))) break;
        if (hipMemcpy(da, e, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    } while (0);
    (void)hipDeviceSynchronize();
    if (hdl) {
        auto destroy = (rocblas_status(*)(rocblas_handle))dlsym(RTLD_DEFAULT,
                                                                 "rocblas_destroy_handle");
        if (destroy) destroy(hdl);
    }
    ba_dfree(buf);
    if (info) ba_dfree(info);
    return rc;
}

int vlgba_mex_bundle_1(int m, int n, int num_a, const double *K, const double *a,
                       const double *b, const double *X, const double *vis, double *X_hat,
                       double *A, double *B, double *e, double *U, double *V, double *W,
                       double *eA, double *eB)
{
    if (num_a == BA_PROJ_NA) return VLGBA_E_NUMA;   // the projective stage has its own entry
    return mex1_impl(VLGBA_MODEL_EUCLIDEAN, m, n, num_a, K, a, b, X, vis, X_hat, A, B, e, U, V,
                     W, eA, eB);
}

int vlgba_mex_bundle_2(int m, int n, int num_a, const double *Y, const double *W,
                       const double *U, const double *eA, const double *eB, double *S,
                       double *e_)
{
    // mex_bundle_2_Se_.c reads num_a = rows(Y) (:57); 12 is the projective twin's
    return mex2_impl(num_a == BA_PROJ_NA ? VLGBA_MODEL_PROJECTIVE : VLGBA_MODEL_EUCLIDEAN, m, n,
                     num_a, Y, W, U, eA, eB, S, e_);
}

int vlgba_mex_bundle_3(int m, int n, int num_a, const double *W, const double *da,
                       const double *eB, const double *Vinv, const double *K, const double *a,
                       const double *b, const double *X, const double *vis, double *db,
                       double *a_new, double *b_new, double *X_hat)
{
    if (num_a == BA_PROJ_NA) return VLGBA_E_NUMA;
    return mex3_impl(VLGBA_MODEL_EUCLIDEAN, m, n, num_a, W, da, eB, Vinv, K, a, b, X, vis, db,
                     a_new, b_new, X_hat);
}

int vlgba_mex_bundle_proj_1(int m, int n, const double *a, const double *b, const double *X,
                            const double *vis, double *X_hat, double *A, double *B, double *e,
                            double *U, double *V, double *W, double *eA, double *eB)
{
    return mex1_impl(VLGBA_MODEL_PROJECTIVE, m, n, BA_PROJ_NA, nullptr, a, b, X, vis, X_hat, A,
                     B, e, U, V, W, eA, eB);
}

int vlgba_mex_bundle_proj_2(int m, int n, const double *Y, const double *W, const double *U,
                            const double *eA, const double *eB, double *S, double *e_)
{
    return mex2_impl(VLGBA_MODEL_PROJECTIVE, m, n, BA_PROJ_NA, Y, W, U, eA, eB, S, e_);
}

int vlgba_mex_bundle_proj_3(int m, int n, const double *W, const double *da, const double *eB,
                            const double *Vinv, const double *a, const double *b,
                            const double *X, const double *vis, double *db, double *a_new,
                            double *b_new, double *X_hat)
{
    return mex3_impl(VLGBA_MODEL_PROJECTIVE, m, n, BA_PROJ_NA, W, da, eB, Vinv, nullptr, a, b, X,
                     vis, db, a_new, b_new, X_hat);
}

}  // extern "C"
