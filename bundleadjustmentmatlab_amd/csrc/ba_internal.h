// ba_internal.h -- device-side data layout and kernel launchers of libvlgba.
//
// One ba_dev per (problem, GPU).  Everything lives in HBM for the whole solve;
// only scalars cross PCIe per LM iteration.  Layout (N = visible observations,
// NA = num_a = 6 / 7 / 10 Euclidean camera parameters or 12 for the projective
// camera P(:) of bundle_projective.m, m cameras, n points):
//
//   observations, point-major (points ascending, cameras ascending inside a
//   point = the reference's column-major (i + n*j) visiting order per point):
//     obs_cam[N] int32, obs_x[N][2] f64, pt_ptr[n+1] int32
//   camera-major view:  cam_ptr[m+1], cam_obs[N] (obs ids ascending)
//   per observation:    jrec[N][JS]   A (2 x NA, column major) then e (2)
//                       W[N][3*NA], Y[N][3*NA]  (NA x 3 column major, as W_ij)
//                       t[N][NA]      Y_o * eB_i (the e_ contribution)
//   per camera:         a[NA*m], a_new, K4[4*m], rot[m][5][9], rot_new[m][5][9],
//                       U[NA*NA*m], eA[NA*m]
//   per point:          b[3n], b_new, V[9n], eB[3n], Vinv[9n], db[3n]
//   reduced system:     blocks (j >= k) with co-visibility: blk_jk[nb][2],
//                       blk_ptr[nb+1], term[T][2] (obs pair, point ascending),
//                       sblk[nb][NA*NA], dense S (NA*m)^2 column major, rhs.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#define VLGBA_CHECK(x)                                                              \
    do {                                                                            \
        hipError_t err__ = (x);                                                     \
        if (err__ != hipSuccess) return -(int)err__;                                \
    } while (0)

// Per-kernel HIP-event timing (diagnostic passes only): every launch of a
// tracked kernel is bracketed by two events on the library stream; after the
// pass the elapsed times are summed per kernel.
enum {
    KT_ROT, KT_LIN, KT_CAMRED, KT_DAMP, KT_SCHUR, KT_SCHUR_CHUNK, KT_SCHUR_RED,
    KT_ASSEMBLE, KT_FACTOR, KT_SYRK, KT_BACKWARD, KT_CAMUPD, KT_PTUPD, KT_CR_FACTOR,
    KT_CR_UPDATE, KT_CR_BACK, KT_SCHUR_MF, KT_LIN_UPD, KT_N
};
#define KT_MAX_EV 8192
struct ba_ktimer {
    int on;
    int nev;
    int ncreated;      // events created so far (on first use: a context that times
                       // few launches creates few)
    hipEvent_t ev[KT_MAX_EV];
    int kid[KT_MAX_EV / 2];
    double ms[KT_N];
    long long calls[KT_N];
    double flops[KT_N];   // the reduced solve's algorithmic flops of the timed passes
};
void kt_begin(struct ba_ktimer *t, hipStream_t s);
void kt_end(struct ba_ktimer *t, hipStream_t s, int kid);

// camera model: NA == BA_PROJ_NA is the projective camera (a = P(:), 3 x 4,
// bundle_projective.m:70-73, projection mex_bundle_proj_1_XABeUVWeAeB.c:13-32;
// no K, no rotations); NA = 6 / 7 / 10 the Euclidean [w; T; (K)]
#define BA_PROJ_NA 12

struct ba_flags {
    int fix_structure;  // V, W, eB = 0       (bundle_euclid.m:140-144)
    int fix_motion;     // U, W, eA = 0       (:145-149)
    int has_pivot;      // pivot[m] mask      (:150-154)
};

// the camera reduction's arguments (k_camera_reduce_chunks, or workgroups
// appended to the MFMA Schur launch)
#ifndef BA_FUSE_CAMRED
#define BA_FUSE_CAMRED 1
#endif
// nested dissection of the envelope: at most this many camera arcs
#ifndef BA_ND_MAX
#define BA_ND_MAX 8
#endif
// ... and at most this many separator tile pairs (their SYRK partials: 33 KB
// each) / host checks (pairs x arc tiles) in its setup, else the natural order
#define BA_ND_MAX_PAIRS 16384LL
#define BA_ND_MAX_SETUP (1LL << 26)
struct ba_camred {
    const int *cam_eptr, *cam_eslots;
    const double *upart;
    int m;
    ba_flags f;
    const unsigned char *pivot;
    double *U, *eA;
    const double *chsse;
    int nch;
    double *sse_out, *sse_out2;
};

struct ba_dev {
    int m, n, na, N, js;
    int device, ncu;   // HIP device ordinal and its CU count
    // problem (read-only)
    int *obs_cam, *pt_ptr, *cam_ptr, *cam_obs;
    double *obs_x, *K4;
    unsigned char *pivot;
    // state
    double *a, *b, *a_new, *b_new;
    double *rot, *rot_new;
    // linearisation
    double *jrec, *W, *U, *eA, *V, *eB;
    // per damping
    double *Vinv, *Y, *t, *db;
    // reduced system
    int nb;            // blocks
    long long T;       // terms
    int *blk_jk, *blk_ptr, *term;
    double *sblk, *rhs, *S, *da;
    long long ld;      // NA*m
    long long lds;     // ld rounded up to the Cholesky tile (padding rows = identity)
    double *linv;      // [lds/64][64*64] inverses of the diagonal Cholesky tiles
    double *ywork;     // [lds] forward-solve result
    // tile envelope of the reduced system (64 x 64 tiles): tile row i of L is
    // non-zero only in tile columns >= tfirst[i] (profile is preserved by the
    // factorisation), so tiles left of it are never touched.
    int nt;
    int *h_tfirst;     // host [nt]
    int *pan_ptr_h;    // host [nt+1]  offsets into pan_list (panel tiles of step k)
    int *h_pan_list;   // host copy of pan_list
    int *pan_list;     // device: tile rows i > k with tfirst[i] <= k, per k
    int *pan_ptr;      // device copy of pan_ptr_h (k_backward_all)
    unsigned long long *xgran64;  // [nt][128] x_k granules of the one-launch backward
    unsigned *kflag;   // [nt] envelope factor: L_kk^-1 / y_k published (epoch fac_epoch)
    unsigned fac_epoch;
    unsigned *rflag;    // [4 nt + 1] runner mode's flags + its timeout word (k_env_runner;
                        // opt-in: VLGBA_ENV_RUNNER=1)
    int env_runner;
    int runner_runs;          // runner launches made (vlgba_plan_info [28])
    int debug_runner_fail;    // the next starts fail (vlgba_debug_force_status word 6)
    hipStream_t rstream;   // the runner's stream (highest priority)
    int *env_tiles;    // device [n_env][2] (i, k) tiles inside the envelope
    int *tb_ptr, *tb_blk;  // device: per envelope tile, the co-visible blocks overlapping it
    int n_env;
    int dense_solve;   // 0 auto, 1: every lower tile (measurement), 2: envelope, no CR,
                       // 3: sequential Cholesky (parity mode), 4: nested dissection
                       // whenever the cameras split (tests; 0 takes it when it pays)
    // block cyclic reduction (tile-tridiagonal S): per level, eliminated tiles
    // (e, p, q) and kept tiles (k, e-, e+, k2); -1 = none
    int cr_nlev;
    int *cr_eptr_h, *cr_kptr_h;   // host [nlev+1]
    int *cr_elim, *cr_keep;       // device [3 * ne], [4 * nk]
    double *crL;                  // [2][nt][64*64] L(p, e) | L(q, e)
    // camera-aligned cyclic reduction: tiles of tb32 = NA * floor(32 / NA)
    // rows (whole cameras, <= 32), padded to 32 in LDS with an identity block;
    // chosen when S is tridiagonal at that granularity (half the pivot chain
    // per level of the 64-row tiles).  crL then holds [2][nt32][32*32] and
    // linv [nt32][32*32].
    int cr32, tb32, nt32;
    // fused levels (L >= 1): records (e, p, q, em, ep) and survivors (k, em, ep)
    int *crf, *crs;               // device
    int *crf_ptr_h, *crs_ptr_h;   // host [nlev + 1], entries per level (level 0 empty)
    // one-launch back substitution (k_cr32_back_all): x of every tile as
    // 64 epoch-tagged 8-byte granules, read by the tiles of the level below
    unsigned long long *xgran;    // [nt32][64]
    unsigned back_epoch;          // per solve, never 0
    // the whole CR in one launch (k_cr32_fused): epoch flags per (level, tile,
    // role 0..2 | survivor); cr_fused = 0 (VLGBA_CR_FUSED=0) keeps the
    // per-level launches
    unsigned *crflag;             // [nlev][nt32][5]
    int cr_fused;
    // direct assembly (camera-aligned CR, one rank, fast path): k_schur_reduce
    // writes each block's lower entries straight into S (and the pinv rule
    // of exactly-zero diagonals), so no k_assemble_tiles launch.  Needs every
    // lower entry of every diagonal CR tile covered by a block (asm_direct_ok,
    // ba_chol_setup): the CR writes only those tiles, so S's other entries
    // keep the zeros of the setup.
    int asm_direct_ok, asm_direct;
    // one-level nested dissection of the envelope (ba_chol_setup, auto mode
    // when S is not tridiagonal; dense_solve 4 forces it): the cameras split
    // into nd_np arcs of consecutive cameras minus the separator (cameras
    // coupled to an earlier arc).  Rows: arc 0 | arc 1 | ... | separator, each
    // part padded to whole 64-row tiles.  Arcs never couple to each other, so
    // step s factors column s of every arc in ONE launch (k_factor_multi);
    // the arcs' contribution to the separator block is one SYRK
    // (k_sep_update / k_sep_reduce), then the separator's columns.
    int nd_np;                    // arcs (0: natural order)
    int nd_grouped;               // k_factor_multi's workgroups grouped by role (nd_step)
    int nd_a0[BA_ND_MAX + 1];     // first tile of arc t; nd_a0[nd_np] = first separator tile
    long long slds;               // rows of the reordered system (nt * 64)
    int *nd_crow;                 // device [m] first row of camera j
    int *nd_prow;                 // device [lds] row of camera-space entry c (-1: padding)
    int *nd_rowsrc;               // device [slds] camera-space entry of row r (-1: padding)
    double *nd_rhs, *nd_x;        // [slds] the rhs / solution in row order
    int nd_npair, nd_nrec;        // separator tile pairs, (pair, arc-column chunk) records
    int *nd_pair;                 // device [npair][2] (i, j), i >= j, ascending
    int *nd_pptr;                 // device [npair + 1] records of each pair
    int *nd_rec;                  // device [nrec][3] (pair, kofs, kcnt)
    int *nd_klist;                // device: the arc columns of the records
    double *nd_part;              // [nrec][64*64 + 64] per-record L_i L_j^T | L_i y
    // algorithmic flops of one reduced solve (ba_chol_setup; bench.py's roofline
    // of the solve kernels): tile-dense potrf + trtri of the diagonal tiles,
    // panel / trailing / fill / SYRK GEMMs and the triangular GEMVs, each counted
    // once (the redundant factorisations of the role-split records are not).
    // fl_factor: the launches timed as k_factor_step / k_cr_factor (with the
    // one-launch CR its back substitution too); fl_syrk: k_sep_update /
    // k_sep_reduce; fl_back: k_backward(_all) / the per-level CR back launches
    double fl_factor, fl_syrk, fl_back;
    // reductions: partial sums per block of the reducing kernels, in fixed order
    double *part;      // [3][PART_MAX]
    double *scal;      // [8] : 0 old_sse, 1 new_sse, 2 dpg cams, 3 dpg pts, 4 non-positive
                       // pivot, 5 hand-off spin timeout (the solve's status words)
    int *chol_cnt;     // arrival counters for the triangular solves
    // ---- fast (chunked) Schur path: points in chunks of <= CH_OBS observations;
    // per chunk the co-visible blocks it touches ("slots") and the cameras it
    // sees ("e-slots") get one partial each, reduced per block in chunk order.
    int ordered;       // 1: sequential bit-exact kernels (k_damp_point + k_schur)
    int parity;        // ordered = 2: + sequential solve and LM scalars (bit-identical
                       // LM trajectory with the oracle)
    ba_camred camred;            // this pass's camera reduction
    int camred_pending;          // ... to run inside the MFMA Schur launch
    int fuse_camred;             // 1: it may (fast path, MFMA groups)
    int mfma;          // fast path: 1 = some MFMA Schur chunks (k_schur_mfma: groups
                       // [0, ngrp_mf)), 0 = term lists only (k_schur_group)
    int no_mfma;       // option: force the term-list Schur kernel
    int ndb;           // camera parameters in the back substitution: 6 (MEX, App. A
                       // Q3) or NA (bundle_euclid_nomex.m semantics)
    int nch;           // chunks
    int *ch_pt;        // [nch+1] local point ranges
    // (the per-chunk slot / term lists stay on the host: they are folded into
    // the chunk records of `blob` and the group-slot lists below)
    int *ch_eslot;     // [nch+1] e-slot ranges
    int *eslot_optr;   // [nes+1]
    unsigned short *eslot_obs;  // [neo] chunk-local obs indices
    int *cam_eptr, *cam_eslots; // per camera: its e-slots in chunk order
    double *spart;     // [ngs][NA*NA] per group slot
    double *epart;     // [nge][NA] per group e-slot
    double *upart;     // [nes][NA(NA+1)/2 + NA] per-chunk U_j (lower) | eA_j partials
    double *chsse;     // [3][nch] per-chunk partials: linearisation SSE, new SSE, point dpg
    // fused update (fast path, ba_launch_update -> k_update_linearize): the
    // next linearisation's buffers, swapped in by an accepted step
    int fused;
    double *W2, *V2, *eB2, *upart2, *chsse2;
    int ns, nes;
    int ch_max_terms, ch_max_slots;   // per-chunk maxima: LDS staging of the term lists
    long long nterm_fast;             // (obs, obs) Schur terms of the chunk plan
    long long blob_words;             // metadata words of the chunk plan
    // Schur groups (consecutive chunks, one workgroup): block / camera partials
    // accumulate in LDS over the group's chunks and are written once per group
    int ngrp, ngs, nge;
    int grp_max_s, grp_max_e;         // LDS accumulator sizes (largest non-direct group)
    unsigned *blob;                   // per-chunk metadata records (see build_plan)
    int *ch_blob, *ch_obase;          // [nch+1] record offsets (words), first local obs
    int *ch_cam;                      // [2 nch] lowest / highest camera of a chunk's obs
    unsigned char *obs_lpt;           // [N] chunk-local point of each observation
    int max_blob;                     // term groups: largest chunk record
    int ngrp_mf;                      // leading MFMA groups
    // long tracks (points [p_long, n), ba_solver.cpp build_plan): segment
    // chunks [nch_reg, nch), their V / eB partials, Schur tiles, update sums
    int nch_reg, nl, p_long;
    int *seg_pt, *seg_long;           // [nch - nch_reg] point, long index
    int *long_pt, *long_o0, *long_seg0;   // [nl], [nl+1] obs range, [nl+1] segments
    int *long_ebase;                  // [nl] first group e-slot
    // per camera its long-track observations in track order (k_schur_reduce
    // merges the lists of a block's two cameras): [m + 1], [nlobs], [nlobs]
    int *cam_lptr, *cam_lobs, *cam_ltrk;
    int max_lcam;                     // longest such list
    int long_o0_h;                    // first long-track observation (host copy)
    double *ylong;                    // [nlobs][3 NA] Y_a = W_a V*^-1 of each long observation
    // per block its long-track terms as (long obs of camera j, of camera k) pairs in
    // track order, found once at setup (k_long_pairs): [nb + 1], [pairs]
    int *lpair_ptr;
    int2 *lpair;
    int *lblk;     // blocks with long-track pairs, most pairs first (k_schur_long_acc)
    int nlb;       // their count (0: k_schur_reduce streams the pairs itself)
    double *vseg;                     // [nseg][12] V | eB partials per segment
    double *dpg_long;                 // [nl] point part of dp'(lambda dp + g)
    int mf_max_s, mf_max_e, mf_max_blob;   // MFMA groups' LDS sizes
    int *grp_ch, *grp_gs, *grp_ge;    // [ngrp+1] chunk / group-slot / group-eslot ranges
    unsigned short *cs_g, *ce_g;      // chunk slot / chunk e-slot -> group-local id
    int *blk_gptr, *blk_gslots;       // per block: its group slots in group order
    int *cam_gptr, *cam_gslots;       // per camera: its group e-slots in group order
    // optional outputs / inputs of the MEX-compatible stage entries (else NULL)
    double *xh_out;    // [N][2] projections (stage 1 and stage 3)
    double *B_out;     // [N][6] point Jacobians (stage 1)
    unsigned char *obs_vis;  // [N] stage 3: 0 = structural-only pair (no projection)
    double red_lambda; // ... at this lambda
    int schur_owner;   // this rank adds U* / eA into the reduced system (every rank
                       // adds its own partials)
    int dpg_lambda;    // this rank adds the lambda dp'dp part of the camera dpg
    double scal_host[8];
    struct ba_ktimer *kt;   // NULL unless kernel timing is enabled
    hipStream_t stream;
    // second stream: the camera reduction runs there, concurrently with V*^-1
    // and the Schur chunks, when the pass is single-rank and untimed;
    // k_schur_reduce (the first consumer of U / eA) waits for ev_join
    hipStream_t side;
    hipEvent_t ev_fork, ev_join;
    int join_pending;
    // host-mapped pass results: [0..5] the scal slots, [7] the pass sequence
    // number written last (k_publish); the host spins on it instead of a
    // device-to-host copy + stream synchronisation
    volatile double *hres;     // host view
    double *hres_dev;          // device view
    unsigned long long seq;
    int publish_req, published;   // fold the publish into the update's final sums
    unsigned *pub_cnt;            // device counter of k_sum_parts3's blocks (zeroed)
};

#define KT_B(d) \
    do { if ((d)->kt && (d)->kt->on) kt_begin((d)->kt, (d)->stream); } while (0)
#define KT_E(d, id) \
    do { if ((d)->kt && (d)->kt->on) kt_end((d)->kt, (d)->stream, (id)); } while (0)

#define BA_PART_MAX 65536
#ifndef BA_CH_OBS
#define BA_CH_OBS 128      // observations per Schur chunk (LDS budget)
#endif
#define BA_CH_PTS 64       // points per Schur chunk
#define BA_CH_TERMS 4096   // (obs, obs) terms per chunk: a track of <= 90 observations
#define BA_GACC 4096       // max doubles of LDS block accumulators per Schur group
#define BA_GE_CAP 128      // cameras per Schur group
#define BA_GROUPS 2048     // target number of Schur groups (workgroups)
#define BA_MF_GROUPS 768   // MFMA Schur groups: one round of 3 workgroups x 256 CUs
#define BA_GROUP_CH 64     // max chunks per Schur group
// MFMA Schur path (k_schur_mfma): a chunk is 4 K-blocks of 5 points (one per
// wave), its cameras span NA * cameras <= 16 * BA_MF_RT slab columns
#define BA_MF_PTS 20
#define BA_MF_RT(na) ((na) == 6 ? 3 : 4)
#define BA_MF_CMAX(na) ((16 * BA_MF_RT(na)) / (na))
#define BA_MF_GACC 1536    // doubles of LDS block accumulators per MFMA Schur group
#define BA_MF_GE_CAP 24    // cameras per MFMA Schur group (LDS budget: 2 groups per CU)
// long tracks (more observations than a chunk holds): segment chunks of
// BA_CH_OBS observations; their Schur terms are added per block by
// k_schur_reduce (merge of the two cameras' long-observation lists).  Caps
// (else the ordered kernels): views per track and (obs, obs) terms of all
// long tracks (the reduce's work)
#define BA_LONG_OBS 65535
#define BA_LONG_TERMS (1LL << 26)
// k_schur_reduce stages a camera's long-observation list in LDS up to this length
#define BA_LCAM_LDS 256
#define BA_LMATCH_BATCH 48   // ... and the matched Y / W rows this many terms at a time

// ---- ba_kernels.hip ----
int ba_launch_rotations(ba_dev *d, const double *a, double *rot, int all5);
int ba_launch_linearize(ba_dev *d, ba_flags f);
// fuse = 1 (an LM pass whose MFMA Schur launch follows): only records the
// reduction for that launch when the plan has MFMA groups
int ba_launch_camera_reduce(ba_dev *d, ba_flags f, int fuse = 0);
int ba_launch_damp_point(ba_dev *d, double lambda);
int ba_launch_schur(ba_dev *d, double lambda);
int ba_launch_assemble(ba_dev *d);
int ba_launch_update(ba_dev *d, double lambda, ba_flags f);
int ba_launch_yeb(ba_dev *d);
int ba_launch_publish(ba_dev *d);   // scal[0..5] + ++seq -> hres (host-mapped)
void *ba_dmalloc(size_t bytes);   // per-device caching allocator (ba_solver.cpp)
// raise kernel fn's dynamic-LDS limit to >= bytes on the current device (cached
// per (kernel, device), thread-safe; ba_solver.cpp)
int ba_ensure_dyn_lds(const void *fn, size_t bytes);
void ba_dfree(void *p);
// after a re-solve: did one of the runner's own hand-offs time out?  Then the
// runner is off for this context (1); 0: no; < 0: error (ba_chol.hip)
int ba_env_runner_timed_out(ba_dev *d);
int ba_launch_schur_fast(ba_dev *d, double lambda);   // fused damp + Vinv + Y + S + e_
// long tracks: count (fill = 0, into cnt[nb]) / write (fill = 1, at lpair_ptr) the
// per-block (obs, obs) pairs of k_schur_reduce (context setup)
int ba_launch_long_pairs(ba_dev *d, int fill, int *cnt);
int ba_launch_assemble_plain(ba_dev *d, double *S, long long ld, int lower_only);
// parity mode (ordered = 2): sequential LM scalars in the reference's flat order
int ba_launch_parity_old_sse(ba_dev *d);
int ba_launch_parity_new_sums(ba_dev *d, double lambda);
// ---- ba_chol.hip ----
int ba_chol_setup(ba_dev *d, const int *blk_jk_host, int nb);
void ba_chol_free(ba_dev *d);
int ba_chol_prepare(ba_dev *d);
int ba_assemble_tiles(ba_dev *d);   // envelope tiles of S + pinv rule + status, one launch
int ba_fix_diag_plain(ba_dev *d, double *S, long long ld);
int ba_chol_fix_diag(ba_dev *d);
// nospin = 1: only launches that never wait on other workgroups (the
// per-level / per-column paths) -- the re-solve after a hand-off timeout
int ba_chol_solve(ba_dev *d, int nospin = 0);
// da = pinv(S) rhs from the eigen-decomposition S = V diag(ev) V^T (ev
// ascending, V column major ld x ld): MATLAB's tolerance ld * eps(max |ev|)
int ba_pinv_apply(ba_dev *d, const double *V, const double *ev, long long ld, const double *rhs,
                  double *work, double *da);

#define TRY_RC(x)                                                                   \
    do {                                                                            \
        int rc__ = (x);                                                             \
        if (rc__) return rc__;                                                      \
    } while (0)
