// Host-side setup of a context, timed on the CPU (no GPU needed): the
// observation sort, the track-kind point order and plan_host (co-visible block
// set + chunk / group plan) of ba_solver.cpp, on a problem read from a file.
// Prints the phase times and an FNV-1a hash of every plan vector, so that a
// reimplementation of the planner can be checked to produce the same plan.
//
// Build (tools/bench_plan.sh): hipcc -O3 -std=c++17 -I include
//   tools/bench_plan.cpp <the library's kernel objects> -lrccl -o tools/build/bench_plan
// Input: int32 m, n, N, then int32 obs_pt[N], int32 obs_cam[N].
#include "../bundleadjustmentmatlab_amd/csrc/ba_solver.cpp"

#include <chrono>
#include <cstdio>

namespace {
struct fnv {
    unsigned long long h = 1469598103934665603ULL;
    template <typename T> void add(const std::vector<T> &v)
    {
        const unsigned char *p = reinterpret_cast<const unsigned char *>(v.data());
        for (size_t q = 0; q < v.size() * sizeof(T); q++) h = (h ^ p[q]) * 1099511628211ULL;
        const unsigned long long n = v.size();
        for (int q = 0; q < 8; q++) h = (h ^ ((n >> (8 * q)) & 0xff)) * 1099511628211ULL;
    }
};
double ms_since(std::chrono::steady_clock::time_point t)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
}  // namespace

int main(int argc, char **argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: bench_plan problem.bin [reps [problem2.bin ...]]\n");
        return 2;
    }
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    // further problem files: planned one after another in this process (the
    // per-thread plan storage reused across different problems, as in a replay)
    for (int fi = 1; fi < argc; fi = (fi == 1 ? 3 : fi + 1)) {
    if (fi >= argc) break;
    FILE *f = std::fopen(argv[fi], "rb");
    if (!f) return 2;
    int hdr[3];
    if (std::fread(hdr, sizeof(int), 3, f) != 3) return 2;
    const int m = hdr[0], n = hdr[1], N = hdr[2];
    std::vector<int> opt(N), ocam(N);
    if (std::fread(opt.data(), sizeof(int), N, f) != (size_t)N ||
        std::fread(ocam.data(), sizeof(int), N, f) != (size_t)N)
        return 2;
    std::fclose(f);
    std::vector<double> ox(2 * (size_t)N, 0.0), K(4 * (size_t)m, 1.0);
    vlgba_problem p{};
    p.m = m;
    p.n = n;
    p.num_a = 6;
    p.num_obs = N;
    p.obs_pt = opt.data();
    p.obs_cam = ocam.data();
    p.obs_x = ox.data();
    p.K = K.data();
    const int na = 6;
    for (int r = 0; r < reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
        host_obs h;
        if (sort_obs(&p, h)) return 3;
        std::vector<int> pt_ptr_all(n + 1, 0);
        for (size_t q = 0; q < h.pt.size(); q++) pt_ptr_all[h.pt[q] + 1]++;
        for (int i = 0; i < n; i++) pt_ptr_all[i + 1] += pt_ptr_all[i];
        const double t_sort = ms_since(t0);
        auto t1 = std::chrono::steady_clock::now();
        std::vector<int> pperm, operm;
        order_points_by_kind(BA_MF_CMAX(na), h, pt_ptr_all, 0, n, pperm, operm);
        std::vector<int> lptr(pt_ptr_all), lcam(h.cam);
        const double t_order = ms_since(t1);
        auto t2 = std::chrono::steady_clock::now();
        bool fast = true;
        int p_long = n;
        // the plan storage as ctx_setup keeps it: per thread, reset per context
        static host_blocks hb;
        static host_plan P;
        hb.reset();
        P.reset();
        plan_host(m, na, n, lptr, lcam, pt_ptr_all, h.cam, 0, n, 0, true, true, false, fast,
                  p_long, hb, P);
        const double t_plan = ms_since(t2);
        {
            auto t3 = std::chrono::steady_clock::now();
            host_blocks hb2;
            build_blocks(m, pt_ptr_all, h.cam, 0, n, 0, true, true, false, hb2);
            std::printf("  build_blocks alone %.2f ms\n", ms_since(t3));
        }
        fnv H;
        H.add(hb.jk);
        H.add(hb.ptr);
        H.add(hb.term);
        H.add(P.ch_pt); H.add(P.ch_slot); H.add(P.ch_eslot); H.add(P.slot_blk);
        H.add(P.slot_tptr); H.add(P.eslot_optr); H.add(P.slot_term); H.add(P.eslot_obs);
        H.add(P.cam_eptr); H.add(P.cam_eslots);
        H.add(P.grp_ch); H.add(P.grp_gs); H.add(P.grp_ge); H.add(P.cs_g); H.add(P.ce_g);
        H.add(P.gslot_blk); H.add(P.gecam); H.add(P.blk_gptr); H.add(P.blk_gslots);
        H.add(P.cam_gptr); H.add(P.cam_gslots); H.add(P.seg_pt); H.add(P.seg_long);
        H.add(P.long_pt); H.add(P.long_o0); H.add(P.long_seg0);
        H.add(P.long_ebase); H.add(P.cam_lptr); H.add(P.cam_lobs); H.add(P.cam_ltrk);
        H.add(P.blob); H.add(P.ch_blob);
        H.add(P.ch_obase);
        const std::vector<int> scal = {P.max_terms, P.max_slots, P.grp_max_s, P.grp_max_e,
                                       P.mf_max_s, P.mf_max_e, P.nch_mf, P.ngrp_mf, P.nch_reg,
                                       P.nseg, P.max_blob, P.mf_max_blob, (int)P.n_terms,
                                       fast ? 1 : 0, p_long};
        H.add(scal);
        {   // MFMA chunk records: camera count and flush flag (ba_solver.cpp build_plan)
            int flush = 0, dense = 0;
            long long csum = 0;
            for (int c = 0; c < P.nch_mf; c++) {
                const unsigned h1 = P.blob[P.ch_blob[c] + 1];
                csum += h1 & 0xffu;
                flush += (h1 >> 9) & 1u;
                dense += (h1 >> 8) & 1u;
            }
            if (P.nch_mf)
                std::printf("  MFMA chunks %d: %.2f cameras each, %d flush (%.1f %%), %d dense\n",
                            P.nch_mf, csum / (double)P.nch_mf, flush, 100.0 * flush / P.nch_mf,
                            dense);
        }
        std::printf("m=%d n=%d N=%d: sort %.2f ms, order %.2f ms, plan_host %.2f ms "
                    "(blocks %d, chunks %zu, groups %zu, blob %zu, fast %d)  hash %016llx\n",
                    m, n, N, t_sort, t_order, t_plan, (int)hb.jk.size() / 2, P.ch_pt.size() - 1,
                    P.grp_ch.size() - 1, P.blob.size(), fast ? 1 : 0, H.h);
    }
    }
    return 0;
}
