// tslam_api.cpp — the C-ABI of libtslam_hip.so (declared in include/tslam.h).
//
// Owns the device workspace of one handle and sequences the stage kernels of a batch on the
// caller's stream.  The launch functions never allocate, copy synchronously or synchronise, so
// a batch can be captured into a hipGraph by the caller.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <limits>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tslam.h"
#include "tslam_ba.h"
#include "tslam_common.h"
#include "tslam_describe.h"
#include "tslam_internal.h"
#include "tslam_tables.h"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace

int tslam_internal_fail(int code, const char* msg) { return fail(code, msg); }

namespace {

#define HIPCHK(expr)                                                                           \
    do {                                                                                       \
        hipError_t e__ = (expr);                                                               \
        if (e__ != hipSuccess)                                                                 \
            return fail(TSLAM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e__));      \
    } while (0)

struct Buffer {
    void* ptr = nullptr;
    int64_t bytes = 0;
    int64_t per_frame = 0;
};
}  // namespace

struct tslam_handle {
    int device = 0;
    tslam_params prm{};
    int W = 0, H = 0, P = 0, C = 0, B = 0, R = 0;
    LevelGeom g{};
    PairCalib calib[8]{};
    uint32_t map_mask = 0;
    int32_t* d_maps = nullptr;
    uint32_t* d_brief = nullptr;
    uint8_t* d_gray = nullptr;   // RGB-D: converted colour images [B][P][H][W]
    // rig pose (tslam_set_rig): E = base_T_rect-left per pair, its inverse, body-frame results
    bool rig = false;
    int rig_q = 0, rig_cap = 0;   // E entries set; allocated
    double* d_rig_E = nullptr;
    double* d_rig_pose = nullptr;
    int32_t* d_rig_stats = nullptr;
    double* d_rig_state = nullptr;
    // IMU rotation prior for the next batch (tslam_set_motion_prior); the rig's body-frame
    // version of it (k_rig_prior), per batch parity
    double* d_prior = nullptr;
    double* d_rig_prior = nullptr;
    hipEvent_t ev_prior[2] = {nullptr, nullptr};   // the last reader of each prior slot is done
    bool prior_read_armed[2] = {false, false};
    bool prior_armed = false;
    double* h_prior_pin[2] = {nullptr, nullptr};   // pinned staging of each parity's prior slot
    bool prior_copy_pending = false;               // copied on the batch's back stream at its first back stage
    // relocalisation map (tslam_map_upload) and scratch
    double* d_map_xyz = nullptr;
    uint32_t* d_map_desc = nullptr;
    int64_t map_n = 0, map_cap = 0;
    int32_t* d_rl_match = nullptr;
    double* d_rl_corr = nullptr;
    int32_t* d_rl_stats = nullptr;
    double* d_rl_pose = nullptr;
    double* d_rl_ransac = nullptr;
    double* d_rl_hyp = nullptr;
    double* d_rl_rig_pose = nullptr;    // tslam_relocalize_rig: the body record
    int32_t* d_rl_rig_stats = nullptr;
    int64_t* d_wedges = nullptr;
    // loop closure (tslam_loop_*): keyframe database, one entry per keyframe, slot = count mod cap
    int lp_cap = 0, lp_S = 0;
    int64_t lp_count = 0;
    double* d_lp_xyz = nullptr;      // [cap][K][3] camera-frame landmarks (compacted)
    uint32_t* d_lp_desc = nullptr;   // [cap][K][8]
    int32_t* d_lp_n = nullptr;       // [cap]
    int32_t* d_lp_votes = nullptr;   // [cap]
    // asynchronous loop closure (tslam_loop_auto / tslam_loop_job_*): keyframes stored by the
    // submit path into entry (k mod cap_k) * P + p with a snapshot of their image; jobs (vote,
    // verify, pose graph) in order on the loop stream, results in pinned memory
    int lp_auto = 0;                       // keyframe interval (0: off)
    int64_t* d_lp_pos = nullptr;           // database positions taken so far (device counter)
    uint32_t* d_lp_snap_kps = nullptr;     // [cap][K][2]
    int32_t* d_lp_snap_kcount = nullptr;   // [cap][TS_MAX_LEVELS]
    uint32_t* d_lp_snap_desc = nullptr;    // [cap][K][8]
    hipStream_t lp_stream = nullptr;
    hipEvent_t lp_ev_store = nullptr;      // the newest batch's keyframe stores (back stream)
    bool lp_store_armed = false;
    struct LoopJob {
        int kind = 0;                      // 0 free, 1 vote, 2 verify, 3 pose graph
        int64_t id = 0;
        hipEvent_t ev = nullptr;
        int n_out = 0, n_edges = 0;        // votes / nodes; pose-graph edges
        void* out = nullptr;               // pinned results
        size_t out_cap = 0;
        void* in = nullptr;                // pinned pose-graph inputs
        size_t in_cap = 0;
        int posted = 0;                    // (worker mutex) 0 queued, 1 on the loop stream, -1 failed
        std::string err;
    } lp_jobs[64];
    int64_t lp_job_next = 1;
    // the loop worker: a host thread that issues the jobs' copies and launches on the loop stream,
    // so a job call returns once its inputs are staged (the caller's frame loop does not pay the
    // ~10-200 launches of a verification or a span solve)
    struct LoopWorker {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        std::deque<std::function<void()>> q;
        int pending = 0;
        bool stop = false;
    }* lp_worker = nullptr;
    // pose graph (tslam_pose_graph) scratch, grown on demand
    int pg_nodes = 0, pg_edges = 0, pg_np = 0;
    double *d_pg_T = nullptr, *d_pg_Z = nullptr, *d_pg_info = nullptr, *d_pg_terms = nullptr;
    double *d_pg_H = nullptr, *d_pg_g = nullptr, *d_pg_delta = nullptr, *d_pg_Ld = nullptr;
    int32_t *d_pg_edges = nullptr, *d_pg_adj_off = nullptr, *d_pg_adj = nullptr, *d_pg_ftile = nullptr;
    double* d_pg_cost = nullptr;   // the solve's cost (k_pg_cost_sum), one double
    // RGB-D dense mapping (tslam_tsdf_*): dense TSDF volume + per-launch pose scratch
    bool tsdf_on = false;
    bool tsdf_color = false;          // colour layer (tslam_tsdf_color)
    TsdfArgs tsdf{};
    double* d_tsdf_poses = nullptr;   // [TSDF_MAX_FRAMES][TSDF_POSE]
    double* d_tsdf_wTc = nullptr;     // [TSDF_MAX_FRAMES][16] host poses staged
    // dense-map outputs (tslam_mesh_* / tslam_esdf_*): scratch sized on first use
    uint8_t* d_mesh_cfg = nullptr;    // [cubes] configuration bytes
    uint32_t* d_mesh_bsum = nullptr;  // [blocks] triangle totals
    uint64_t* d_mesh_boff = nullptr;  // [blocks] first triangle; [blocks] = mesh total
    size_t mesh_cubes_cap = 0;
    float* d_mesh_tris = nullptr;     // [tri cap][9]
    float* d_mesh_cols = nullptr;     // [tri cap][9] vertex colours (colour layer)
    int64_t mesh_tris_cap = 0, mesh_n = 0;
    int32_t* d_edt[2] = {nullptr, nullptr};
    size_t edt_cap = 0;
    float* d_esdf = nullptr;          // [nz][ny][nx]
    size_t esdf_cap = 0;
    bool esdf_valid = false;
    float* d_dist_tab = nullptr;      // [R^2 + 1]
    int dist_tab_R = -1;
    double dist_tab_s = 0.0;
    uint8_t* d_slice_obs = nullptr;
    float* d_slice = nullptr;
    size_t slice_cap = 0;
    Buffer buf[TSLAM_BUF_COUNT];
    uint32_t* d_cand = nullptr;
    uint32_t* d_ccount = nullptr;
    uint32_t* d_det_thr_acc = nullptr;   // [C][L] running minimum of the next te
    uint32_t* d_hist = nullptr;
    double* d_state = nullptr;
    double* d_ransac = nullptr;
    double* d_hyp = nullptr;
    int64_t frames_done = 0;
    // current batch
    const uint8_t* cur_images = nullptr;
    int cur_n = 0;
    int64_t cur_g0 = 0;
    bool in_batch = false;
    hipStream_t last_stream = nullptr;
    std::vector<void*> allocs;
    // A8 keyframe window (slots shared by all pairs: keyframes are whole frames)
    BaStore ba{};
    int64_t ba_frame[TS_BA_MAXW]{};
    int64_t ba_nkf = 0;
    int64_t ba_last = -1;    // newest frame inserted
    BaTiming ba_timing{};    // k_ba_schur events while profiling is on
    bool ba_split = false;   // tslam_ba_split_solve: k_ba_reduce + k_ba_solve instead of k_ba_reduce_solve
    // tslam_ba_defer: a BA stage on its own stream is enqueued later (the next batch's first back
    // stage, or any call that reads or changes BA state), so the caller's next front stages are on
    // the GPU before this batch's ~160 BA launches are issued from the host
    bool ba_defer = false;
    struct {
        bool pending = false;
        BatchCtx c{};
        hipStream_t s = nullptr;
        double* snap = nullptr;
        double* snap_body = nullptr;
        int32_t* assoc = nullptr;
        int par = 0;
    } ba_job;
    std::map<std::pair<int, int64_t>, std::array<double, 10>> ba_imu;   // (pair, keyframe) -> IMU factor
    // (pair, keyframe) -> inertial factor record + initial velocity (tslam_ba_inertial_factor)
    std::map<std::pair<int, int64_t>, std::array<double, TS_BA_INE + 3>> ba_ine;
    std::vector<std::array<double, 12>> ba_icfg;            // per pair: gravity, bias priors and weights (BaArgs.icfg)
    std::vector<std::array<uint8_t, TS_BA_MAXW>> ba_ine_slot;   // per pair and slot: carries a factor
    std::vector<BaArgs> ba_solved;   // per pair: the arguments of its last window solve (replays)
    // A pair window's keyframe chain (eviction, gate, tiles, iters x (Schur, reduce-and-solve),
    // back substitution: ~16 launches) replayed from a captured hipGraph per chain shape: the
    // kernels read a device record (BaRec) written by the graph's first node, so a replay costs one
    // node update and one graph launch instead of ~16 launches with 2 KB of by-value arguments.
    // Each shape keeps a ring of instances (own record, event of its last replay), so an instance
    // is updated only once its previous replay has run.
    struct BaGraphInst {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        hipGraphNode_t setrec = nullptr;
        hipEvent_t done = nullptr;
        bool armed = false;
        BaRec* d_rec = nullptr;
    };
    struct BaGraphSet {
        std::array<int, 6> key{};   // evict, eviction n_order, n_order, inertial, split, iters
        std::vector<BaGraphInst> inst;
        int next = 0;
    };
    // tslam_ba_graph: off by default — measured on MI355X (tools/ba_probe.py), a
    // replay (one node update + the graph launch) costs the host 162 us per keyframe against 80 us
    // for the 16 direct launches, and the chain's GPU time 0.240 against 0.222 ms
    bool ba_graph = false;
    std::vector<BaGraphSet> ba_graphs;
    hipStream_t ba_cap_stream = nullptr;
    // BA on its own stream (overlapping the next batch): events and the batch parity
    int64_t batch_idx = 0;
    bool batch_started = false;
    hipStream_t ba_stream = nullptr;
    hipEvent_t ev_fe = nullptr, ev_ba[2] = {nullptr, nullptr};
    bool ba_pending[2] = {false, false};
    // front (rectify .. describe) and back (match .. chain) stages on two streams: batch s's back
    // waits for its front; batch s's front waits for the back of batch s - 2 (shared ring slots)
    hipStream_t front_stream = nullptr, back_stream = nullptr;
    bool front_started = false, back_started = false;
    hipEvent_t ev_front = nullptr, ev_back[2] = {nullptr, nullptr};
    bool back_pending[2] = {false, false};
    std::vector<hipEvent_t> ba_events;
    // sharded rig (tslam_set_shard): front-end cameras [sh_cam_lo, sh_cam_hi) and back-end frames
    // [rank * n / world, (rank + 1) * n / world) of every batch
    int sh_cam_lo = 0, sh_cam_hi = 0, sh_rank = 0, sh_world = 1;
    // pair split (TSLAM_SHARD_PAIRS, one camera per rank): the back end solves this camera's pair
    // over half of the batch and the rig pose covers range rig_slot (tslam_ranges.h)
    bool sh_pairs = false;
    // library-driven sharding (tslam_comm_init / tslam_group_create, tslam_shard.cpp): the driver
    // that owns this rank's communicators, streams and exchange buffers (owned here after
    // tslam_comm_init; a group owns it otherwise)
    bool sh_comm = false;
    tslam_shard_driver* drv = nullptr;
    bool drv_owned = false;
    // asynchronous host boundary (tslam_submit_host / tslam_poll_*): the handle's own front/back
    // streams, pinned staging + device input per batch parity, pinned result slots per parity
    hipStream_t as_front = nullptr, as_back = nullptr;
    hipStream_t as_ba = nullptr;      // local BA (ba_window > 0): its own stream on every CU
    uint8_t* as_stage[2] = {nullptr, nullptr};   // pinned host
    uint8_t* as_input[2] = {nullptr, nullptr};   // device
    hipEvent_t as_staged[2] = {nullptr, nullptr};   // DMA out of as_stage[k] done
    bool as_staged_armed[2] = {false, false};
    struct ResultSlot {
        double* pose = nullptr;       // pinned [B][P][68]
        int32_t* stats = nullptr;     // pinned [B][P][8]
        double* rig_pose = nullptr;   // pinned [B][68]
        int32_t* rig_stats = nullptr; // pinned [B][8]
        std::vector<double> ts;
        hipEvent_t ev = nullptr;
        int64_t batch = -1, g0 = 0;
        int n = 0;
        bool pending = false;         // completed or in flight, not yet returned by tslam_poll_batch
    } as_res[2];
    int64_t as_batches = 0;           // batches submitted through tslam_submit_host
    int64_t as_last_pose_batch = -1;  // newest batch tslam_poll_pose returned
    std::vector<void*> host_allocs;
};

static int dev_alloc(tslam_handle* h, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(TSLAM_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    h->allocs.push_back(*p);
    HIPCHK(hipMemset(*p, 0, bytes));
    // hipMemset is ordered on the null stream only: the handle's non-blocking streams (and the
    // caller's) could otherwise write the buffer before the zeroing lands on it
    HIPCHK(hipDeviceSynchronize());
    return TSLAM_OK;
}

// release *p (if any) and allocate `bytes` fresh (zeroed)
static int dev_realloc(tslam_handle* h, void** p, size_t bytes) {
    if (*p) {
        (void)hipFree(*p);
        h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), *p), h->allocs.end());
        *p = nullptr;
    }
    return dev_alloc(h, p, bytes);
}

static void free_all(tslam_handle* h) {
    if (h->drv && h->drv_owned) tslam_internal_driver_destroy(h->drv);
    h->drv = nullptr;
    for (void* p : h->allocs) (void)hipFree(p);
    h->allocs.clear();
    for (void* p : h->host_allocs) (void)hipHostFree(p);
    h->host_allocs.clear();
}

// -- the loop worker (tslam_loop_job_*) -----------------------------------------------------------
static void loop_worker_run(tslam_handle* h) {
    auto* w = h->lp_worker;
    (void)hipSetDevice(h->device);
    for (;;) {
        std::function<void()> f;
        {
            std::unique_lock<std::mutex> lk(w->mu);
            w->cv.wait(lk, [&] { return w->stop || !w->q.empty(); });
            if (w->q.empty()) return;
            f = std::move(w->q.front());
            w->q.pop_front();
        }
        f();
        {
            std::lock_guard<std::mutex> lk(w->mu);
            --w->pending;
        }
        w->cv.notify_all();
    }
}

static void loop_worker_post(tslam_handle* h, std::function<void()> f) {
    if (!h->lp_worker) {
        h->lp_worker = new tslam_handle::LoopWorker();
        h->lp_worker->th = std::thread(loop_worker_run, h);
    }
    {
        std::lock_guard<std::mutex> lk(h->lp_worker->mu);
        h->lp_worker->q.push_back(std::move(f));
        ++h->lp_worker->pending;
    }
    h->lp_worker->cv.notify_all();
}

// every posted job is on the loop stream
static void loop_worker_drain(tslam_handle* h) {
    if (!h->lp_worker) return;
    std::unique_lock<std::mutex> lk(h->lp_worker->mu);
    h->lp_worker->cv.wait(lk, [&] { return h->lp_worker->pending == 0; });
}

static void loop_worker_stop(tslam_handle* h) {
    if (!h->lp_worker) return;
    {
        std::lock_guard<std::mutex> lk(h->lp_worker->mu);
        h->lp_worker->stop = true;
    }
    h->lp_worker->cv.notify_all();
    h->lp_worker->th.join();   // the queue is drained first (the thread exits on an empty queue)
    delete h->lp_worker;
    h->lp_worker = nullptr;
}

static void build_geometry(tslam_handle* h) {
    LevelGeom& g = h->g;
    const tslam_params& p = h->prm;
    g.n_levels = p.n_levels;
    g.K = p.n_features;
    int w = h->W, hh = h->H, off = 0;
    double tot = 0.0;
    for (int l = 0; l < p.n_levels; ++l) tot += std::pow(0.25, l);
    int sumq = 0;
    for (int l = 0; l < p.n_levels; ++l) {
        g.W[l] = w;
        g.H[l] = hh;
        g.pyr_off[l] = off;
        off += w * hh;
        w >>= 1;
        hh >>= 1;
        g.Kq[l] = (int)((double)p.n_features * std::pow(0.25, l) / tot);
        if (l > 0) sumq += g.Kq[l];
    }
    g.Kq[0] = p.n_features - sumq;
    g.pyr_bytes = (off + 15) & ~15;
    int ko = 0, bs = 0, co = 0, qs = 0;
    // detect band height at level 0: the tallest of 32 / 24 / 16 rows whose band (2 * rows + 10
    // rows of W bytes of LDS) keeps 3 (W <= 640) or 2 (W <= 1280) blocks per CU; measured 778 ->
    // 690 us at 640x400 (32 rows) and 611 -> 575 us at 1280x800 (24 rows) against 16.  Coarser
    // levels take taller bands in the same LDS budget (fewer blocks and halo rows, similar pixels
    // per block), equalised over the level's rows: 640x400 -> 32 / 68 / 100 / 50 rows, 26 -> 18
    // blocks per image, 662 -> 625 us per 256-frame batch
    const int br0 = (2 * TS_BAND_ROWS_MAX + 10) * g.W[0] <= 48 * 1024 ? TS_BAND_ROWS_MAX
                  : (2 * 24 + 10) * g.W[0] <= 78 * 1024 ? 24 : 16;
    const int det_budget = (2 * br0 + 10) * g.W[0];
    g.det_lds = 0;
    for (int l = 0; l < p.n_levels; ++l) {
        // <= 124 rows: detect's phase-B queue entries hold the score row (< 128) in 7 bits and the
        // quad (< 512, so W <= 2044) in 9
        const int maxr = l == 0 ? br0 : std::max(br0, std::min(124, (det_budget / g.W[l] - 10) / 2));
        const int nb = (g.H[l] + maxr - 1) / maxr;
        g.band_rows[l] = l == 0 ? br0 : ((g.H[l] + nb - 1) / nb + 1) & ~1;
        g.smooth_groups[l] = std::max(2, g.band_rows[l] / 16);
        g.det_lds = std::max(g.det_lds, (2 * g.band_rows[l] + 10) * g.W[l]);
    }
    g.dt_total = 0;
    for (int l = 0; l < p.n_levels; ++l) {
        g.koff[l] = ko;
        ko += g.Kq[l];
        g.nbands[l] = (g.H[l] + g.band_rows[l] - 1) / g.band_rows[l];
        g.band_start[l] = bs;
        bs += g.nbands[l];
        g.cand_cap[l] = ((g.band_rows[l] + 1) / 2) * (g.W[l] / 2 + 1);
        g.cand_off[l] = co;
        co += g.nbands[l] * g.cand_cap[l];
        g.dt_nx[l] = (g.W[l] + TS_DT_W - 1) / TS_DT_W;
        g.dt_start[l] = g.dt_total;
        g.dt_total += g.dt_nx[l] * ((g.H[l] + TS_DT_H - 1) / TS_DT_H);
        g.qtiles[l] = (g.Kq[l] + 127) / 128;   // k_match: TS_MQ queries per block
        g.qtile_start[l] = qs;
        qs += g.qtiles[l];
    }
    g.total_bands = bs;
    g.cand_total = co;
    g.total_qtiles = qs;
    int ro = 0;
    for (int l = 0; l < p.n_levels; ++l) {
        g.rs_off[l] = ro;
        ro += g.H[l] + 1;
    }
    g.rs_total = (ro + 7) & ~7;
}

// Storage pairs of A8: the P stereo pairs plus pair P, the body window of the rig-level solve
// (tslam_ba.h); every storage pair has its own solve scratch (strides as in ba_pair).
static int alloc_ba(tslam_handle* h) {
    const size_t W = h->prm.ba_window, K = h->g.K, P = h->P + 1, WK = W * K, M = TS_BA_MAXW;
    BaStore& b = h->ba;
    struct A {
        void** p;
        size_t bytes;
    } list[] = {
        {(void**)&b.T, 8 * P * W * 16},      {(void**)&b.Tfe, 8 * P * W * 16},   {(void**)&b.u, 8 * P * WK},
        {(void**)&b.v, 8 * P * WK},          {(void**)&b.d, 8 * P * WK},         {(void**)&b.lm, 4 * P * WK},
        {(void**)&b.X, 8 * P * WK * 3},      {(void**)&b.kf_desc, 32 * P * WK},  {(void**)&b.gid, 8 * P * WK},
        {(void**)&b.remap, 4 * P * K},       {(void**)&b.cnt, 4 * P * WK},
        {(void**)&b.lm_id, 4 * P * WK},      {(void**)&b.keep, P * WK},          {(void**)&b.obs_Vg, 8 * P * WK * 9},
        {(void**)&b.lmask, 4 * P * (WK / 32 + 64)}, {(void**)&b.lpre, 4 * P * (WK / 32 + 64)},
        {(void**)&b.tc_fl, P * TS_BA_TILES * 256},  {(void**)&b.tc_ids, 4 * P * TS_BA_TILES * 2048},
        {(void**)&b.cam_off, 4 * P * (W + 1)},
        {(void**)&b.counts, 4 * 4 * P},      {(void**)&b.tiles, 4 * P * 2 * TS_BA_TILES}, {(void**)&b.done, 4 * P},
        {(void**)&b.lo_o, 4 * P * WK * M},   {(void**)&b.lo_uvd, 32 * P * WK * M}, {(void**)&b.lo_W, 8 * 18 * P * WK * M},
        {(void**)&b.Xc, 8 * P * WK * 3},
        {(void**)&b.lm_L, 8 * P * WK * 6},   {(void**)&b.lm_gp, 8 * P * WK * 3}, {(void**)&b.C, 8 * P * 64 * 64},
        {(void**)&b.part, 8 * P * (size_t)TS_BA_SPLIT * TS_BA_PART}, {(void**)&b.cam_U, 8 * P * W * 27}, {(void**)&b.dc, 8 * P * W * 6},
        {(void**)&b.flops, 8},               {(void**)&b.fe_pose, 8 * 2 * (size_t)h->B * h->P * 16},
        {(void**)&b.fe_body, 8 * 2 * (size_t)h->B * 16}, {(void**)&b.imu, 8 * P * W * 10},
        {(void**)&b.kf_assoc, 4 * 2 * (size_t)h->B * h->P * K},
        {(void**)&b.ine, 8 * P * W * TS_BA_INE}, {(void**)&b.vel, 8 * P * W * 3}, {(void**)&b.bias, 8 * P * W * 6},
    };
    for (const A& a : list) {
        const int rc = dev_alloc(h, a.p, a.bytes);
        if (rc != TSLAM_OK) return rc;
    }
    // scratch kept in its between-solves state by the kernels themselves (no per-solve memsets):
    // the slot table all -1 (k_ba_insert_gate clears the rows the last solve filled), remap all
    // 0x7F7F7F7F (k_ba_insert refills it after an eviction), cnt zero (dev_alloc; k_ba_backsub
    // re-zeroes it)
    HIPCHK(hipMemset(b.lo_o, 0xFF, 4 * P * WK * M));
    HIPCHK(hipMemset(b.remap, 0x7F, 4 * P * K));
    HIPCHK(hipDeviceSynchronize());
    h->ba_icfg.assign(h->P + 1, std::array<double, 12>{});   // pair windows + a rig's body window
    h->ba_ine_slot.assign(h->P + 1, std::array<uint8_t, TS_BA_MAXW>{});
    return TSLAM_OK;
}

static BaArgs ba_args(tslam_handle* h) {
    BaArgs a{};
    a.st = h->ba;
    a.W = h->prm.ba_window;
    a.interval = h->prm.ba_kf_interval;
    a.iters = h->prm.ba_iters;
    a.nsplit = TS_BA_SPLIT;
    a.lam = h->prm.ba_lambda;
    a.outlier_px = h->prm.ba_outlier_px;
    a.prev = -1;
    return a;
}

// Occupied slots, oldest keyframe first, without `skip`.
static int ba_order(const tslam_handle* h, int skip, int* out) {
    int n = 0;
    for (int s = 0; s < h->prm.ba_window; ++s)
        if (h->ba_frame[s] >= 0 && s != skip) out[n++] = s;
    std::sort(out, out + n, [h](int a, int b) { return h->ba_frame[a] < h->ba_frame[b]; });
    return n;
}

static BatchCtx make_ctx(tslam_handle* h);

// Rig-level A8: a handle with tslam_set_rig over several pairs solves one body window.
static bool ba_rig(const tslam_handle* h) { return h->rig && h->P > 1 && h->prm.ba_window; }

static constexpr int BA_GRAPH_MAX = 32;   // instances per chain shape (keyframes of that shape in flight)

// One pair window's keyframe chain through the graph cache (see BaGraphInst): a finished instance
// of the chain's shape is re-pointed at this keyframe's record, a new one is captured only while
// every instance still has a replay in flight (the steady state needs two or three per shape).
static hipError_t ba_chain_graph(tslam_handle* h, const BaRec& r, bool evict, bool split, bool ine, hipStream_t s) {
    const std::array<int, 6> key{evict ? 1 : 0, evict ? r.evict.n_order : 0, r.a.n_order, ine ? 1 : 0, split ? 1 : 0,
                                 r.a.iters};
    tslam_handle::BaGraphSet* set = nullptr;
    for (auto& g : h->ba_graphs)
        if (g.key == key) set = &g;
    if (!set) {
        h->ba_graphs.emplace_back();
        set = &h->ba_graphs.back();
        set->key = key;
    }
    hipError_t e = hipSuccess;
    const int n = (int)set->inst.size();
    int pick = -1;
    for (int k = 0; k < n && pick < 0; ++k) {   // round robin from the oldest replay
        const int i = (set->next + k) % n;
        tslam_handle::BaGraphInst& in = set->inst[(size_t)i];
        if (!in.armed) {
            pick = i;
        } else {
            e = hipEventQuery(in.done);
            if (e == hipSuccess) pick = i;
            else if (e != hipErrorNotReady) return e;
        }
    }
    if (pick < 0 && n == BA_GRAPH_MAX) {   // every instance busy: wait for the oldest replay
        pick = set->next % n;
        if ((e = hipEventSynchronize(set->inst[(size_t)pick].done)) != hipSuccess) return e;
    }
    if (pick < 0) {   // a new instance: capture the chain on a private stream (nothing runs), instantiate it
        tslam_handle::BaGraphInst in;
        if (dev_alloc(h, (void**)&in.d_rec, sizeof(BaRec)) != TSLAM_OK) return hipErrorOutOfMemory;
        if (!h->ba_cap_stream && (e = hipStreamCreateWithFlags(&h->ba_cap_stream, hipStreamNonBlocking)) != hipSuccess)
            return e;
        if ((e = hipStreamBeginCapture(h->ba_cap_stream, hipStreamCaptureModeThreadLocal)) != hipSuccess) return e;
        launch_ba_setrec(r, in.d_rec, h->ba_cap_stream);
        launch_ba_chain_rec(r, in.d_rec, evict, split, ine, h->ba_cap_stream);
        if ((e = hipStreamEndCapture(h->ba_cap_stream, &in.graph)) != hipSuccess) return e;
        size_t n_root = 1;
        if ((e = hipGraphGetRootNodes(in.graph, &in.setrec, &n_root)) != hipSuccess) return e;
        if (n_root != 1) return hipErrorInvalidValue;
        if ((e = hipGraphInstantiate(&in.exec, in.graph, nullptr, nullptr, 0)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&in.done, hipEventDisableTiming)) != hipSuccess) return e;
        set->inst.push_back(in);
        pick = n;
    } else if ((e = ba_graph_set_record(set->inst[(size_t)pick].exec, set->inst[(size_t)pick].setrec, r,
                                        set->inst[(size_t)pick].d_rec)) != hipSuccess) {
        return e;
    }
    tslam_handle::BaGraphInst& in = set->inst[(size_t)pick];
    set->next = (pick + 1) % (int)set->inst.size();
    if ((e = hipGraphLaunch(in.exec, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(in.done, s)) != hipSuccess) return e;
    in.armed = true;
    return hipSuccess;
}

static void ba_graphs_destroy(tslam_handle* h) {
    for (auto& g : h->ba_graphs)
        for (auto& in : g.inst) {
            if (in.exec) (void)hipGraphExecDestroy(in.exec);
            if (in.graph) (void)hipGraphDestroy(in.graph);
            if (in.done) (void)hipEventDestroy(in.done);
        }
    h->ba_graphs.clear();
    if (h->ba_cap_stream) (void)hipStreamDestroy(h->ba_cap_stream);
    h->ba_cap_stream = nullptr;
}

// A8: every keyframe of the current batch (g % ba_kf_interval == 0) enters each pair's window,
// evicting the oldest when the window is full, and the window is solved (per pair, or for a rig
// one joint body solve: launch_ba_rig_solve).  Host bookkeeping of the slots only; nothing
// synchronises.  `fe_body`: the rig front end's snapshot of the batch (rig-level A8).
static hipError_t run_ba(tslam_handle* h, const BatchCtx& c, hipStream_t s, const double* fe, const double* fe_body,
                         const int32_t* kf_assoc) {
    const int W = h->prm.ba_window, iv = h->prm.ba_kf_interval;
    // pair windows replay their keyframe chains from graphs (not while Schur launches are timed)
    const bool graph = h->ba_graph && !ba_rig(h) && !h->ba_timing.ev;
    std::vector<BaArgs> ev_args;
    for (int64_t g = c.g0; g < c.g0 + c.n; ++g) {
        if (g % iv != 0 || g <= h->ba_last) continue;
        BaArgs a = ba_args(h);
        a.fe = fe;
        a.kf_assoc = kf_assoc;
        a.frame = g;
        a.slot = (int)(h->ba_nkf % W);
        int ord[TS_BA_MAXW];
        const int nocc = ba_order(h, -1, ord);
        a.prev = nocc ? ord[nocc - 1] : -1;
        const bool evict = h->ba_frame[a.slot] >= 0;
        if (evict) a.n_order = ba_order(h, a.slot, a.order);
        const bool rig = ba_rig(h);
        if (rig) {   // the body pose first, every pair's camera E_p^-1 B (and the body's inertial factor)
            a.fe_body = fe_body;
            a.pose_given = 1;
            auto jt = h->ba_ine.find({h->P, g});
            const bool has = jt != h->ba_ine.end();
            for (int e = 0; e < TS_BA_INE; ++e) a.ine[e] = has ? jt->second[e] : 0.0;
            for (int e = 0; e < 3; ++e) a.vel0[e] = has ? jt->second[TS_BA_INE + e] : 0.0;
            if (has) h->ba_ine.erase(jt);
            h->ba_ine_slot[h->P][a.slot] = has && a.ine[28] > 0.0;
            launch_ba_rig_keyframe(c, a, s);
        }
        // per pair: the keyframe's IMU rotation factor, inertial factor and initial velocity (zero
        // for a rig's pairs), inserted by the solve's first launch (k_ba_insert_gate)
        std::vector<std::array<double, 10 + TS_BA_INE + 3>> kfi((size_t)h->P);
        for (int p = 0; p < h->P; ++p) {
            a.pair = p;
            auto& v = kfi[(size_t)p];
            auto it = h->ba_imu.find({p, g});   // the keyframe's IMU rotation factor (if given)
            for (int e = 0; e < 10; ++e) v[e] = (!rig && it != h->ba_imu.end()) ? it->second[e] : 0.0;
            if (it != h->ba_imu.end()) h->ba_imu.erase(it);
            auto jt = h->ba_ine.find({p, g});   // and its inertial factor + initial velocity
            const bool has = !rig && jt != h->ba_ine.end();
            for (int e = 0; e < TS_BA_INE + 3; ++e) v[10 + e] = has ? jt->second[e] : 0.0;
            if (jt != h->ba_ine.end()) h->ba_ine.erase(jt);
            h->ba_ine_slot[p][a.slot] = has && v[10 + 28] > 0.0;
            if (graph)
                ev_args.push_back(a);   // the eviction runs first in the pair's chain below
            else
                launch_ba_keyframe(c, a, evict, s);   // eviction only
        }
        for (int e = 0; e < 10; ++e) a.imu[e] = 0.0;
        for (int e = 0; e < TS_BA_INE; ++e) a.ine[e] = 0.0;
        for (int e = 0; e < 3; ++e) a.vel0[e] = 0.0;
        for (auto it = h->ba_imu.begin(); it != h->ba_imu.end();)   // factors of frames already past
            it = it->first.second < g ? h->ba_imu.erase(it) : std::next(it);
        for (auto it = h->ba_ine.begin(); it != h->ba_ine.end();)
            it = it->first.second < g ? h->ba_ine.erase(it) : std::next(it);
        h->ba_frame[a.slot] = g;
        h->ba_nkf += 1;
        h->ba_last = g;
        a.n_order = ba_order(h, -1, a.order);
        h->ba_solved.resize(h->P);
        if (rig) {
            for (int e = 0; e < 12; ++e) a.icfg[e] = h->ba_icfg[h->P][e];
            bool ine = false;
            for (int k = 1; k < a.n_order; ++k) ine = ine || h->ba_ine_slot[h->P][a.order[k]];
            launch_ba_rig_solve(c, a, s, h->ba_timing.ev ? &h->ba_timing : nullptr, ine);
            for (int p = 0; p < h->P; ++p) {
                h->ba_solved[p] = a;
                h->ba_solved[p].pair = p;
            }
            continue;
        }
        for (int p = 0; p < h->P; ++p) {
            a.pair = p;
            const auto& v = kfi[(size_t)p];
            for (int e = 0; e < 10; ++e) a.imu[e] = v[e];
            for (int e = 0; e < TS_BA_INE; ++e) a.ine[e] = v[10 + e];
            for (int e = 0; e < 3; ++e) a.vel0[e] = v[10 + TS_BA_INE + e];
            for (int e = 0; e < 12; ++e) a.icfg[e] = h->ba_icfg[p][e];
            // the inertial kernels when a factor links two keyframes of the window (the oldest
            // keyframe's factor points out of it)
            bool ine = false;
            for (int k = 1; k < a.n_order; ++k) ine = ine || h->ba_ine_slot[p][a.order[k]];
            if (graph) {
                const BaRec r{c, ev_args[(size_t)p], a};
                const hipError_t e = ba_chain_graph(h, r, evict, h->ba_split, ine, s);
                if (e != hipSuccess) return e;
            } else {
                launch_ba_solve(c, a, s, h->ba_timing.ev ? &h->ba_timing : nullptr, h->ba_split, ine);
            }
            h->ba_solved[p] = a;
        }
        if (graph) ev_args.clear();
    }
    return hipSuccess;
}

static BatchCtx make_ctx(tslam_handle* h) {
    BatchCtx c{};
    c.g = h->g;
    c.C = h->C;
    c.P = h->P;
    c.B = h->B;
    c.R = h->R;
    c.n = h->cur_n;
    c.g0 = h->cur_g0;
    c.W = h->W;
    c.H = h->H;
    c.cpp = h->prm.rgbd ? 1 : 2;
    c.rgbd = h->prm.rgbd;
    c.images = h->prm.rgbd ? h->d_gray : h->cur_images;
    c.rgbd_in = h->prm.rgbd ? h->cur_images : nullptr;
    c.maps = h->d_maps;
    c.map_mask = h->map_mask;
    c.pyr = (uint8_t*)h->buf[TSLAM_BUF_PYRAMID].ptr;
    c.smo = (uint8_t*)h->buf[TSLAM_BUF_SMOOTH].ptr;
    c.cand = h->d_cand;
    c.ccount = h->d_ccount;
    c.hist = h->d_hist;
    c.kps = (uint32_t*)h->buf[TSLAM_BUF_KEYPOINTS].ptr;
    c.kcount = (int32_t*)h->buf[TSLAM_BUF_KCOUNT].ptr;
    c.desc = (uint32_t*)h->buf[TSLAM_BUF_DESC].ptr;
    c.ys = (uint4*)h->buf[TSLAM_BUF_YSORTED].ptr;
    c.desc_ys = (uint32_t*)h->buf[TSLAM_BUF_DESC_YS].ptr;
    c.rowstart = (uint16_t*)h->buf[TSLAM_BUF_ROWSTART].ptr;
    c.qbest = (uint32_t*)h->buf[TSLAM_BUF_QBEST].ptr;
    c.qsecond = (uint32_t*)h->buf[TSLAM_BUF_QSECOND].ptr;
    c.tbest = (uint32_t*)h->buf[TSLAM_BUF_TBEST].ptr;
    c.stereo = (int32_t*)h->buf[TSLAM_BUF_STEREO].ptr;
    c.disp = (double*)h->buf[TSLAM_BUF_DISP].ptr;
    c.temporal = (int32_t*)h->buf[TSLAM_BUF_TEMPORAL].ptr;
    c.tuv = (double*)h->buf[TSLAM_BUF_TEMPORAL_UV].ptr;
    c.corr = (double*)h->buf[TSLAM_BUF_CORR].ptr;
    c.pose = (double*)h->buf[TSLAM_BUF_POSE].ptr;
    c.stats = (int32_t*)h->buf[TSLAM_BUF_STATS].ptr;
    c.state = h->d_state;
    c.prior = h->prior_armed ? h->d_prior + (size_t)(h->batch_idx & 1) * TS_PRIOR_DOUBLES * h->P * h->B : nullptr;
    c.rig_E = h->d_rig_E;
    c.rig_Einv = h->d_rig_E ? h->d_rig_E + 16 * h->rig_q : nullptr;
    c.rig_pose = h->d_rig_pose;
    c.rig_stats = h->d_rig_stats;
    c.rig_state = h->d_rig_state;
    c.rig_prior = (h->prior_armed && h->d_rig_prior) ? h->d_rig_prior + (size_t)(h->batch_idx & 1) * TS_PRIOR_DOUBLES * h->B
                                                     : nullptr;
    c.ransac = h->d_ransac;
    c.hyp = h->d_hyp;
    c.det_thr = (const uint32_t*)h->buf[TSLAM_BUF_DET_THR].ptr;
    c.det_thr_acc = h->d_det_thr_acc;
    c.det_fail = (uint32_t*)h->buf[TSLAM_BUF_DET_FAIL].ptr;
    c.brief_table = h->d_brief;
    c.wedges = h->d_wedges;
    for (int p = 0; p < h->P; ++p) c.calib[p] = h->calib[p];
    c.mp.max_hamming = h->prm.max_hamming;
    c.mp.ratio_pct = h->prm.ratio_pct;
    c.mp.row_tol = h->prm.stereo_row_tol;
    c.mp.max_disp = h->prm.max_disparity;
    c.mp.window = h->prm.temporal_window;
    c.pp.n_hyp = h->prm.ransac_hypotheses;
    c.pp.iters = h->prm.refine_iters;
    c.pp.min_inliers = h->prm.min_inliers;
    c.pp.splits = h->prm.ransac_splits;
    c.pp.mode = h->prm.ransac_mode;
    c.pp.refine_block = h->prm.refine_block;
    c.pp.thr2 = h->prm.ransac_thr_px * h->prm.ransac_thr_px;
    c.pp.seed = h->prm.ransac_seed;
    c.fast_threshold = h->prm.fast_threshold;
    c.margin = h->prm.edge_margin;
    c.cam0 = h->sh_cam_lo;
    c.ncam = h->sh_cam_hi - h->sh_cam_lo;
    c.pair0 = 0;
    c.npair = h->P;
    c.match_modes = 3;
    c.reloc = 0;
    c.peer_S = c.peer_me = c.peer_nbuf = c.peer_skip = 0;
    return c;
}

// The back-end context of batch frames [lo, hi): frame lo is the context's frame 0 and every
// batch-indexed buffer is offset to batch frame lo, so results land where a whole-batch run puts
// them (ring-indexed buffers need no offset: they are addressed by global frame).
static BatchCtx range_ctx(const BatchCtx& c, int lo, int hi) {
    BatchCtx r = c;
    const size_t P = c.P, K = c.g.K, f = lo;
    r.g0 = c.g0 + lo;
    r.n = hi - lo;
    r.qbest += f * P * 2 * K;
    r.qsecond += f * P * 2 * K;
    r.tbest += f * P * 2 * K;
    r.tuv += f * P * K * 2;
    r.corr += f * P * K * TS_CORR_DOUBLES;
    r.pose += f * P * TS_POSE_DOUBLES;
    r.stats += f * P * TS_STATS_INTS;
    r.ransac += f * P * TS_MAX_SPLITS * TS_RANSAC_WORDS / 2;
    r.hyp += f * P * 4 * (size_t)c.pp.n_hyp * TS_HYP_DOUBLES;
    if (r.prior) r.prior += f * P * TS_PRIOR_DOUBLES;
    if (r.rig_prior) r.rig_prior += f * TS_PRIOR_DOUBLES;
    if (r.rig_pose) r.rig_pose += f * TS_POSE_DOUBLES;
    if (r.rig_stats) r.rig_stats += f * TS_STATS_INTS;
    return r;
}

// the rank's rig range: rig pose, pose records (and, without the pair split, its whole back end)
static void shard_range(const tslam_handle* h, int n, int* lo, int* hi) {
    peer_range(rig_slot(h->sh_rank, h->sh_world, h->sh_pairs), n, h->sh_world, lo, hi);
}
// pair split: the half of the batch whose frames this rank's pair back end solves
static void pair_half(const tslam_handle* h, int n, int* lo, int* hi) { peer_range(h->sh_cam_lo & 1, n, 2, lo, hi); }

// A8 of the current batch.  It may run on its own stream: it depends on this batch's poses (event
// on the stream of the last stage) and only reads ring buffers plus a snapshot of the batch's
// poses, so the next batch can start.  A sharded rank runs it once its ring holds every pair's
// keyframe data (rank 0 after the state gather, tslam_shard.cpp).
// The deferred BA job (tslam_ba_defer): its stream already waits for its batch's back end, so
// issuing it later only moves the host work.
static int ba_flush(tslam_handle* h) {
    if (!h->ba_job.pending) return TSLAM_OK;
    h->ba_job.pending = false;
    auto& j = h->ba_job;
    HIPCHK(hipSetDevice(h->device));   // flushed from any entry point, before it sets the device
    hipError_t e = run_ba(h, j.c, j.s, j.snap, j.snap_body, j.assoc);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(h->ev_ba[j.par], j.s);
    if (e != hipSuccess) {   // no event to wait for: the window's state is unknown, say so now
        h->ba_pending[j.par] = false;
        return fail(TSLAM_EHIP, std::string("deferred BA: ") + hipGetErrorString(e));
    }
    return TSLAM_OK;
}
#define BA_FLUSH(h)                                    \
    do {                                               \
        if ((h) && (h)->ba_job.pending) {              \
            const int rc_flush__ = ba_flush(h);        \
            if (rc_flush__ != TSLAM_OK) return rc_flush__; \
        }                                              \
    } while (0)

static int ba_stage(tslam_handle* h, const BatchCtx& c, hipStream_t s) {
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    BA_FLUSH(h);   // the previous batch's deferred BA comes first (host state, event order)
    const int par = (int)(h->batch_idx & 1);
    double* snap = h->ba.fe_pose + (size_t)par * h->B * h->P * 16;
    double* snap_body = h->ba.fe_body + (size_t)par * h->B * 16;
    int32_t* assoc = h->ba.kf_assoc + (size_t)par * h->B * h->P * h->g.K;
    hipStream_t fs = h->last_stream;
    launch_ba_snapshot(c, snap, fs);
    launch_ba_kf_assoc(c, assoc, h->prm.ba_kf_interval, fs);
    if (ba_rig(h)) launch_ba_snapshot_rig(c, snap_body, fs);
    const bool other = s != fs;
    if (other) {
        if (!h->ev_fe) {
            HIPCHK(hipEventCreateWithFlags(&h->ev_fe, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&h->ev_ba[0], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&h->ev_ba[1], hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(h->ev_fe, fs));
        HIPCHK(hipStreamWaitEvent(s, h->ev_fe, 0));
        if (h->ba_defer) {   // enqueued at the next flush point (BA_FLUSH)
            h->ba_job.pending = true;
            h->ba_job.c = c;
            h->ba_job.s = s;
            h->ba_job.snap = snap;
            h->ba_job.snap_body = snap_body;
            h->ba_job.assoc = assoc;
            h->ba_job.par = par;
            h->ba_pending[par] = true;
            return TSLAM_OK;
        }
    }
    if (const hipError_t e = run_ba(h, c, s, snap, snap_body, assoc); e != hipSuccess)
        return fail(TSLAM_EHIP, std::string("BA: ") + hipGetErrorString(e));
    if (other) {
        HIPCHK(hipEventRecord(h->ev_ba[par], s));
        h->ba_pending[par] = true;
    }
    return TSLAM_OK;
}

// Stages of a sharded handle (tslam_set_shard, world > 1).  Front stages run on the handle's
// cameras for every frame of the batch; back stages on the rank's frame range [lo, hi) of the
// batch, after the exchange has filled the other cameras' ring slots for frames lo-1 .. hi-1:
// MATCH first re-derives the stereo disparities of frame lo-1 (the range's first frame
// triangulates from them; the rank that owns lo-1 computes the same values), POSE adds the rig
// pose of the range (no chaining), and CHAIN chains the whole batch once every rank's pose
// records are back (tslam_unpack_poses), identically on every rank.
//
// A camera-sharded RGB-D rig (each camera is a "pair": its back end needs no other camera) instead
// tracks its own cameras over the whole batch: MATCH and POSE run on the pair view of its cameras
// for every frame; the rig pose of its frame range (KERNEL_RIG) follows tslam_unpack_pairs of the
// other ranks' pair blocks (pose, stats, correspondences); then pose records and CHAIN as above.
static int run_sharded_rgbd_stage(tslam_handle* h, const BatchCtx& c, int stage, hipStream_t s) {
    int lo, hi;
    shard_range(h, c.n, &lo, &hi);
    BatchCtx own = c;   // pair view: this rank's cameras (cameras per pair = 1)
    own.pair0 = h->sh_cam_lo;
    own.npair = h->sh_cam_hi - h->sh_cam_lo;
    switch (stage) {
        case TSLAM_STAGE_RECTIFY:
        case TSLAM_KERNEL_RECTIFY_PYRAMID:
            launch_rgbd_gray(c, h->d_gray, s);
            launch_rectify_pyramid(c, s);
            break;
        case TSLAM_STAGE_DETECT: launch_detect(c, s); launch_select(c, s); break;
        case TSLAM_STAGE_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_KERNEL_DETECT: launch_detect(c, s); break;
        case TSLAM_KERNEL_SELECT: launch_select(c, s); break;
        case TSLAM_KERNEL_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_STAGE_MATCH: launch_match(own, s); launch_match_refine(own, s); break;
        case TSLAM_KERNEL_MATCH: launch_match(own, s); break;
        case TSLAM_KERNEL_MATCH_REFINE: launch_match_refine(own, s); break;
        case TSLAM_STAGE_POSE:
        case TSLAM_KERNEL_POSE: launch_pose(own, s); break;
        case TSLAM_KERNEL_RIG:
            if (!h->rig) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
            if (hi > lo) launch_rig_pose(range_ctx(c, lo, hi), s);
            break;
        case TSLAM_KERNEL_CHAIN: launch_chains(c, h->rig, s); break;
        default:
            return fail(TSLAM_ESTATE, "a camera-sharded RGB-D handle runs its stages one by one: RECTIFY..DESCRIBE, "
                                      "MATCH, POSE, pack/exchange/unpack pairs, KERNEL_RIG, pose records, CHAIN");
    }
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

static int run_sharded_stage(tslam_handle* h, const BatchCtx& c, int stage, hipStream_t s) {
    if (h->prm.rgbd) return run_sharded_rgbd_stage(h, c, stage, s);
    int lo, hi;
    if (h->sh_pairs) pair_half(h, c.n, &lo, &hi);
    else shard_range(h, c.n, &lo, &hi);
    BatchCtx cb = range_ctx(c, lo, hi);
    const bool empty = hi <= lo;           // a short batch leaves this rank no frames
    const bool pre = !empty && c.g0 + lo - 1 >= 0;   // frame lo - 1 exists
    BatchCtx cp = c;                        // the pre-pass: frame lo - 1, batch scratch at frame 0
    cp.g0 = c.g0 + lo - 1;
    cp.n = 1;
    if (h->sh_pairs) {   // pair split: this camera's pair only; the rig pose is its own step (KERNEL_RIG)
        cb.pair0 = cp.pair0 = h->sh_cam_lo / 2;
        cb.npair = cp.npair = 1;
        switch (stage) {
            case TSLAM_STAGE_POSE:
                if (!empty) launch_pose(cb, s);
                HIPCHK(hipGetLastError());
                return TSLAM_OK;
            case TSLAM_KERNEL_RIG: {
                if (!h->rig) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
                int rl, rh;
                shard_range(h, c.n, &rl, &rh);   // every pair's blocks of the rig range are here (tslam_shard.cpp)
                if (rh > rl) launch_rig_pose(range_ctx(c, rl, rh), s);
                HIPCHK(hipGetLastError());
                return TSLAM_OK;
            }
            default: break;
        }
    }
    switch (stage) {
        case TSLAM_STAGE_RECTIFY: launch_rectify_pyramid(c, s); break;
        case TSLAM_STAGE_DETECT: launch_detect(c, s); launch_select(c, s); break;
        case TSLAM_STAGE_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_KERNEL_RECTIFY_PYRAMID: launch_rectify_pyramid(c, s); break;
        case TSLAM_KERNEL_DETECT: launch_detect(c, s); break;
        case TSLAM_KERNEL_SELECT: launch_select(c, s); break;
        case TSLAM_KERNEL_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_STAGE_MATCH:
            if (pre) launch_match_stereo(cp, s);
            if (!empty) {
                launch_match(cb, s);
                launch_match_refine(cb, s);
            }
            break;
        case TSLAM_KERNEL_MATCH:
            if (pre) launch_match_stereo(cp, s);
            if (!empty) launch_match(cb, s);
            break;
        case TSLAM_KERNEL_MATCH_REFINE:
            if (!empty) launch_match_refine(cb, s);
            break;
        case TSLAM_STAGE_POSE:
            if (!empty) launch_pose(cb, s);
            if (!empty && h->rig) launch_rig_pose(cb, s);
            break;
        case TSLAM_KERNEL_POSE:
            if (!empty) launch_pose(cb, s);
            break;
        case TSLAM_KERNEL_RIG:
            if (!h->rig) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
            if (!empty) launch_rig_pose(cb, s);
            break;
        case TSLAM_KERNEL_CHAIN: launch_chains(c, h->rig, s); break;
        case TSLAM_STAGE_BA: return ba_stage(h, c, s);   // rank 0 of a gathering driver
        default:
            return fail(TSLAM_ESTATE, "a sharded handle runs its stages one by one around the exchange "
                                      "(RECTIFY..DESCRIBE, pack/exchange/unpack, MATCH, POSE, exchange, CHAIN)");
    }
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

extern "C" {

const char* tslam_last_error(void) { return g_err.c_str(); }

int tslam_abi_version(void) { return TSLAM_ABI_VERSION; }

int tslam_create(const tslam_stereo_desc* pairs, const tslam_params* params, int device, tslam_handle** out) {
    if (!pairs || !params || !out) return fail(TSLAM_EINVAL, "null argument");
    const tslam_params& p = *params;
    if (p.n_pairs < 1 || p.n_pairs > 8) return fail(TSLAM_EINVAL, "n_pairs must be in [1, 8]");
    if (p.n_levels < 1 || p.n_levels > TS_MAX_LEVELS) return fail(TSLAM_EINVAL, "n_levels must be in [1, 6]");
    if (p.n_features < 1 || p.n_features > 8192) return fail(TSLAM_EINVAL, "n_features must be in [1, 8192]");
    if (p.ransac_hypotheses < 1 || p.ransac_hypotheses > 256) return fail(TSLAM_EINVAL, "ransac_hypotheses must be in [1, 256]");
    if (p.edge_margin < 19) return fail(TSLAM_EINVAL, "edge_margin must be >= 19");
    if (p.fast_threshold < 0 || p.fast_threshold > 254) return fail(TSLAM_EINVAL, "fast_threshold must be in [0, 254]");
    if (p.max_batch < 1) return fail(TSLAM_EINVAL, "max_batch must be >= 1");
    if (p.max_hamming < 0 || p.max_hamming > 253) return fail(TSLAM_EINVAL, "max_hamming must be in [0, 253]");
    // k_match packs the gate offsets into 16-bit halves (query xy + window < 2^15)
    if (p.stereo_row_tol < 0 || p.stereo_row_tol > 2047 || p.max_disparity < 0 || p.max_disparity > 2047 ||
        p.temporal_window < 0 || p.temporal_window > 2047)
        return fail(TSLAM_EINVAL, "stereo_row_tol, max_disparity, temporal_window must be in [0, 2047]");
    if (!(p.ba_window == 0 || (p.ba_window >= 2 && p.ba_window <= TS_BA_MAXW)))
        return fail(TSLAM_EINVAL, "ba_window must be 0 (off) or in [2, 10]");
    if (p.ba_window && (p.ba_kf_interval < 1 || p.ba_iters < 1 || !(p.ba_lambda >= 0.0) || !(p.ba_outlier_px > 0.0)))
        return fail(TSLAM_EINVAL, "ba_kf_interval, ba_iters >= 1, ba_lambda >= 0, ba_outlier_px > 0");
    if (p.refine_iters < 1) return fail(TSLAM_EINVAL, "refine_iters must be >= 1");
    if (p.ransac_splits < 0 || p.ransac_splits > TS_MAX_SPLITS) return fail(TSLAM_EINVAL, "ransac_splits must be in [0, 32]");
    if (p.ransac_mode < 0 || p.ransac_mode > 2) return fail(TSLAM_EINVAL, "ransac_mode must be 0, 1 or 2");
    if (p.refine_block != 0 && p.refine_block != 128 && p.refine_block != 256)
        return fail(TSLAM_EINVAL, "refine_block must be 0, 128 or 256");
    const int W = pairs[0].width, H = pairs[0].height;
    if (W < 64 || H < 64 || W > 2047 || H > 2047) return fail(TSLAM_EINVAL, "image size must be within [64, 2047]");
    for (int i = 1; i < p.n_pairs; ++i)
        if (pairs[i].width != W || pairs[i].height != H) return fail(TSLAM_EINVAL, "all pairs must share the image size");
    if ((H >> (p.n_levels - 1)) < 2 * p.edge_margin + 3 || (W >> (p.n_levels - 1)) < 2 * p.edge_margin + 3)
        return fail(TSLAM_EINVAL, "coarsest pyramid level smaller than 2*edge_margin+3");
    for (int i = 0; i < p.n_pairs; ++i)
        if (!(p.rgbd || pairs[i].baseline > 0.0) || !(pairs[i].fx > 0.0) || !(pairs[i].fy > 0.0))
            return fail(TSLAM_EINVAL, "pair calibration needs fx, fy, baseline > 0");
    if (p.rgbd != 0 && p.rgbd != 1) return fail(TSLAM_EINVAL, "rgbd must be 0 or 1");
    if (p.rgbd && ((W * H) & 1)) return fail(TSLAM_EINVAL, "RGB-D needs an even pixel count (u16 depth alignment)");

    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(TSLAM_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(e));

    tslam_handle* h = new tslam_handle();
    h->device = device;
    h->prm = p;
    h->W = W;
    h->H = H;
    h->P = p.n_pairs;
    h->C = (p.rgbd ? 1 : 2) * p.n_pairs;
    h->B = p.max_batch;
    h->sh_cam_hi = h->C;
    // the ring keeps frame t-1 of a batch's first frame; with BA it also keeps the frames a
    // keyframe's temporal match chain walks back over
    // the ring keeps frame t-1 of a batch's first frame while the front stages of the next batch
    // run (front / back on two streams): R = 2B + 1
    h->R = 2 * p.max_batch + 1;
    // with BA the ring also keeps the frames a keyframe's match chain walks back over, even while
    // the next batch runs (BA may run on its own stream): R = 2B + interval + 1
    if (p.ba_window) h->R = 2 * p.max_batch + p.ba_kf_interval + 1;
    build_geometry(h);
    for (int i = 0; i < h->P; ++i) {
        h->calib[i].fx = pairs[i].fx;
        h->calib[i].fy = pairs[i].fy;
        h->calib[i].cx = pairs[i].cx;
        h->calib[i].cy = pairs[i].cy;
        h->calib[i].fxb = pairs[i].fx * (p.rgbd ? 1.0 : pairs[i].baseline);   // RGB-D: virtual 1 m baseline
    }

    const int64_t K = p.n_features, C = h->C, P = h->P, B = h->B, R = h->R, L = p.n_levels;
    struct Spec {
        int which;
        int64_t frames;
        int64_t per_frame;
    } specs[] = {
        {TSLAM_BUF_PYRAMID, R, C * h->g.pyr_bytes},
        {TSLAM_BUF_SMOOTH, B, C * h->g.pyr_bytes},
        {TSLAM_BUF_KEYPOINTS, R, C * K * 2 * 4},
        {TSLAM_BUF_KCOUNT, R, C * L * 4},
        {TSLAM_BUF_DESC, R, C * K * 8 * 4},
        {TSLAM_BUF_STEREO, R, P * K * 4},
        {TSLAM_BUF_DISP, R, P * K * 8},
        {TSLAM_BUF_TEMPORAL, R, P * K * 4},
        {TSLAM_BUF_TEMPORAL_UV, B, P * K * 2 * 8},
        {TSLAM_BUF_CORR, B, P * K * TS_CORR_DOUBLES * 8},
        {TSLAM_BUF_POSE, B, P * TS_POSE_DOUBLES * 8},
        {TSLAM_BUF_STATS, B, P * TS_STATS_INTS * 4},
        {TSLAM_BUF_QBEST, B, P * 2 * K * 4},
        {TSLAM_BUF_QSECOND, B, P * 2 * K * 4},
        {TSLAM_BUF_TBEST, B, P * 2 * K * 4},
        {TSLAM_BUF_YSORTED, R, C * K * 16},
        {TSLAM_BUF_DESC_YS, R, C * K * 8 * 4},
        {TSLAM_BUF_ROWSTART, R, C * (int64_t)h->g.rs_total * 2},
        {TSLAM_BUF_DET_THR, 1, C * L * 4},
        {TSLAM_BUF_DET_FAIL, B, C * L * 4},
        {TSLAM_BUF_HYP, B, P * 4 * (int64_t)p.ransac_hypotheses * TS_HYP_DOUBLES * 8},
    };
    int rc = TSLAM_OK;
    for (const Spec& s : specs) {
        Buffer& b = h->buf[s.which];
        b.per_frame = s.per_frame;
        b.bytes = s.per_frame * s.frames;
        if ((rc = dev_alloc(h, &b.ptr, (size_t)b.bytes)) != TSLAM_OK) break;
    }
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_cand, sizeof(uint32_t) * (size_t)B * C * h->g.cand_total);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_ccount, sizeof(uint32_t) * (size_t)B * C * h->g.total_bands);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_hist, sizeof(uint32_t) * (size_t)B * C * L * 256);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_det_thr_acc, sizeof(uint32_t) * (size_t)C * L);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_state, sizeof(double) * 32 * (size_t)P);   // chain (A, Q) per pair
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_ransac, sizeof(uint32_t) * TS_RANSAC_WORDS * TS_MAX_SPLITS * (size_t)B * P);
    if (rc == TSLAM_OK) h->d_hyp = (double*)h->buf[TSLAM_BUF_HYP].ptr;
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_brief, sizeof(TSLAM_BRIEF_TABLE));
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_wedges, sizeof(TSLAM_WEDGES));
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_maps, sizeof(int32_t) * (size_t)C * W * H * 2);
    if (rc == TSLAM_OK && p.ba_window) rc = alloc_ba(h);
    if (rc == TSLAM_OK && p.rgbd) rc = dev_alloc(h, (void**)&h->d_gray, (size_t)B * P * W * H);
    if (rc != TSLAM_OK) {
        free_all(h);
        delete h;
        return rc;
    }
    // the describe kernel reads the rotated pattern as byte offsets from the patch origin
    // (x - 18, y - 18) in its LDS tile: (py + 18) * TS_DT_P + px + 18 for both points, packed
    // low | high << 16
    std::vector<uint32_t> brief_off(30 * 256);
    for (int i = 0; i < 30 * 256; ++i) {
        const uint32_t t = TSLAM_BRIEF_TABLE[i];
        const int px = (int8_t)(t & 0xFF), py = (int8_t)((t >> 8) & 0xFF);
        const int qx = (int8_t)((t >> 16) & 0xFF), qy = (int8_t)(t >> 24);
        brief_off[i] = (uint32_t)((py + 18) * TS_DT_P + px + 18) | ((uint32_t)((qy + 18) * TS_DT_P + qx + 18) << 16);
    }
    bool ok = hipMemcpy(h->d_brief, brief_off.data(), sizeof(uint32_t) * brief_off.size(), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(h->d_wedges, TSLAM_WEDGES, sizeof(TSLAM_WEDGES), hipMemcpyHostToDevice) == hipSuccess;
    for (int i = 0; i < h->P && ok; ++i) {
        const int32_t* m[2] = {pairs[i].map_left, pairs[i].map_right};
        const int cpp = p.rgbd ? 1 : 2;
        for (int s = 0; s < cpp; ++s) {
            if (!m[s]) continue;
            h->map_mask |= 1u << (cpp * i + s);
            ok = ok && hipMemcpy(h->d_maps + (size_t)(cpp * i + s) * W * H * 2, m[s], sizeof(int32_t) * (size_t)W * H * 2,
                                 hipMemcpyHostToDevice) == hipSuccess;
        }
    }
    if (!ok) {
        free_all(h);
        delete h;
        return fail(TSLAM_EHIP, "uploading tables / maps failed");
    }
    if (tslam_reset(h) != TSLAM_OK) {
        free_all(h);
        delete h;
        return TSLAM_EHIP;
    }
    *out = h;
    return TSLAM_OK;
}

int tslam_destroy(tslam_handle* h) {
    if (!h) return TSLAM_OK;
    (void)ba_flush(h);   // destroyed whatever the deferred BA reports
    loop_worker_stop(h);   // its queued jobs reach the loop stream before the device is drained
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : h->ba_events) (void)hipEventDestroy(e);
    for (auto& j : h->lp_jobs)
        if (j.ev) (void)hipEventDestroy(j.ev);
    if (h->lp_ev_store) (void)hipEventDestroy(h->lp_ev_store);
    if (h->lp_stream) (void)hipStreamDestroy(h->lp_stream);
    for (hipEvent_t e : {h->ev_fe, h->ev_ba[0], h->ev_ba[1], h->ev_front, h->ev_back[0], h->ev_back[1], h->ev_prior[0],
                         h->ev_prior[1],
                         h->as_staged[0], h->as_staged[1], h->as_res[0].ev, h->as_res[1].ev})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t st : {h->as_front, h->as_back, h->as_ba})
        if (st) (void)hipStreamDestroy(st);
    ba_graphs_destroy(h);
    free_all(h);
    delete h;
    return TSLAM_OK;
}

int tslam_reset(tslam_handle* h) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    loop_worker_drain(h);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<double> eye(32 * (size_t)h->P, 0.0);   // every chain's (A, Q) = (I, I)
    for (int q = 0; q < 2 * h->P; ++q)
        for (int k = 0; k < 4; ++k) eye[(size_t)q * 16 + 5 * k] = 1.0;
    HIPCHK(hipMemcpy(h->d_state, eye.data(), sizeof(double) * eye.size(), hipMemcpyHostToDevice));
    if (h->d_rig_state) HIPCHK(hipMemcpy(h->d_rig_state, eye.data(), sizeof(double) * 32, hipMemcpyHostToDevice));
    h->frames_done = 0;
    // the speculative FAST threshold starts exact (t + 1) and learns from the first batch
    HIPCHK(hipMemset(h->buf[TSLAM_BUF_DET_THR].ptr, 0, sizeof(uint32_t) * (size_t)h->C * h->g.n_levels));
    HIPCHK(hipMemset(h->d_det_thr_acc, 0xFF, sizeof(uint32_t) * (size_t)h->C * h->g.n_levels));
    for (int i = 0; i < TS_BA_MAXW; ++i) h->ba_frame[i] = -1;
    h->ba_nkf = 0;
    h->ba_last = -1;
    h->ba_solved.clear();
    if (h->prm.ba_window) {   // the inertial state of the window belongs to the session
        const size_t P = h->P + 1, W = h->prm.ba_window;
        HIPCHK(hipMemset(h->ba.ine, 0, 8 * P * W * TS_BA_INE));
        HIPCHK(hipMemset(h->ba.vel, 0, 8 * P * W * 3));
        HIPCHK(hipMemset(h->ba.bias, 0, 8 * P * W * 6));
        h->ba_ine.clear();
        h->ba_imu.clear();
        for (auto& f : h->ba_ine_slot) f.fill(0);
    }
    if (h->tsdf_on) {   // so does the dense map
        const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
        HIPCHK(hipMemset(h->tsdf.tsdf, 0, sizeof(float) * nv));
        HIPCHK(hipMemset(h->tsdf.weight, 0, sizeof(float) * nv));
        if (h->tsdf.col) {
            HIPCHK(hipMemset(h->tsdf.col, 0, sizeof(float) * 3 * nv));
            HIPCHK(hipMemset(h->tsdf.col_w, 0, sizeof(float) * nv));
        }
    }
    h->lp_count = 0;   // the keyframe database belongs to the session
    if (h->d_lp_n) HIPCHK(hipMemset(h->d_lp_n, 0, sizeof(int32_t) * (size_t)h->lp_cap));   // every entry empty
    if (h->d_lp_pos) HIPCHK(hipMemset(h->d_lp_pos, 0, sizeof(int64_t)));
    for (auto& j : h->lp_jobs) j.kind = 0;   // jobs of the old session are dropped
    h->lp_store_armed = false;
    h->ba_pending[0] = h->ba_pending[1] = false;
    h->back_pending[0] = h->back_pending[1] = false;
    h->in_batch = false;
    h->cur_n = 0;
    for (auto& r : h->as_res) r.pending = false;   // results of batches before the reset are dropped
    h->as_last_pose_batch = h->as_batches - 1;
    // hipMemset runs on the null stream, which the handle's non-blocking streams do not wait for
    HIPCHK(hipDeviceSynchronize());
    return TSLAM_OK;
}

// -- asynchronous host boundary -------------------------------------------------------------------
static int64_t host_frame_bytes(const tslam_handle* h) {
    return h->prm.rgbd ? (int64_t)h->P * 5 * h->W * h->H : (int64_t)h->C * h->W * h->H;
}

// pinned result slots per batch parity (tslam_poll_batch / tslam_poll_pose read them)
static int ensure_result_slots(tslam_handle* h) {
    if (h->as_res[0].ev) return TSLAM_OK;
    const size_t B = h->B, P = h->P;
    for (int k = 0; k < 2; ++k) {
        auto& r = h->as_res[k];
        const size_t bytes[4] = {8 * B * P * TS_POSE_DOUBLES, 4 * B * P * TS_STATS_INTS, 8 * B * TS_POSE_DOUBLES,
                                 4 * B * TS_STATS_INTS};
        void** dst[4] = {(void**)&r.pose, (void**)&r.stats, (void**)&r.rig_pose, (void**)&r.rig_stats};
        for (int i = 0; i < 4; ++i) {
            HIPCHK(hipHostMalloc(dst[i], bytes[i], hipHostMallocDefault));
            h->host_allocs.push_back(*dst[i]);
        }
        r.ts.assign(B, 0.0);
        HIPCHK(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
    }
    return TSLAM_OK;
}

static int ensure_async(tslam_handle* h) {
    if (h->as_front) return TSLAM_OK;
    int rc = ensure_result_slots(h);
    if (rc != TSLAM_OK) return rc;
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    if (h->prm.ba_window) {
        // local BA: its chain of small dependent launches (one-block solves, ~135-block Schur
        // passes) runs on a stream of its own, and the front / back kernels stay off the last
        // TS_BA_CU_RESERVE CUs so those launches find free CUs beside the next batch's front end
        // (C4: 15.1k -> 16.2k frames/s, bench.py --front-cu-reserve sweep)
        int n_cu = 0;
        HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, h->device));
        const int keep = n_cu > 2 * TS_BA_CU_RESERVE ? n_cu - TS_BA_CU_RESERVE : n_cu;
        std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
        for (int cu = 0; cu < keep; ++cu) mask[(size_t)cu / 32] |= 1u << (cu % 32);
        HIPCHK(hipExtStreamCreateWithCUMask(&h->as_front, (uint32_t)mask.size(), mask.data()));
        HIPCHK(hipExtStreamCreateWithCUMask(&h->as_back, (uint32_t)mask.size(), mask.data()));
        HIPCHK(hipStreamCreateWithPriority(&h->as_ba, hipStreamNonBlocking, hi));
    } else {
        HIPCHK(hipStreamCreateWithPriority(&h->as_front, hipStreamNonBlocking, hi));   // front = critical path
        HIPCHK(hipStreamCreateWithFlags(&h->as_back, hipStreamNonBlocking));
    }
    const size_t in_bytes = (size_t)h->B * host_frame_bytes(h);
    for (int k = 0; k < 2; ++k) {
        void* p = nullptr;
        HIPCHK(hipHostMalloc(&p, in_bytes, hipHostMallocDefault));
        h->host_allocs.push_back(p);
        h->as_stage[k] = (uint8_t*)p;
        rc = dev_alloc(h, (void**)&h->as_input[k], in_bytes);
        if (rc != TSLAM_OK) return rc;
        HIPCHK(hipEventCreateWithFlags(&h->as_staged[k], hipEventDisableTiming));
    }
    return TSLAM_OK;
}

// The current batch's results into the pinned slot of its parity on stream s (an unread batch s-2
// there is dropped), for tslam_poll_batch / tslam_poll_pose.  Timestamps: `ts` or frame indices.
static int stash_results(tslam_handle* h, const double* ts, hipStream_t s) {
    int rc = ensure_result_slots(h);
    if (rc != TSLAM_OK) return rc;
    const int k = (int)(h->as_batches & 1);
    auto& r = h->as_res[k];
    const size_t n = h->cur_n, P = h->P;
    HIPCHK(hipMemcpyAsync(r.pose, h->buf[TSLAM_BUF_POSE].ptr, 8 * n * P * TS_POSE_DOUBLES, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(r.stats, h->buf[TSLAM_BUF_STATS].ptr, 4 * n * P * TS_STATS_INTS, hipMemcpyDeviceToHost, s));
    if (h->rig) {
        HIPCHK(hipMemcpyAsync(r.rig_pose, h->d_rig_pose, 8 * n * TS_POSE_DOUBLES, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(r.rig_stats, h->d_rig_stats, 4 * n * TS_STATS_INTS, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipEventRecord(r.ev, s));
    for (size_t i = 0; i < n; ++i) r.ts[i] = ts ? ts[i] : (double)(h->cur_g0 + (int64_t)i);
    r.batch = h->as_batches;
    r.g0 = h->cur_g0;
    r.n = (int)n;
    r.pending = true;
    h->as_batches += 1;
    return TSLAM_OK;
}

int tslam_host_stage(tslam_handle* h, uint8_t** stage, int64_t* frame_bytes) {
    if (!h || !stage) return fail(TSLAM_EINVAL, "bad argument");
    if (h->sh_world > 1 || h->sh_comm) return fail(TSLAM_ESTATE, "a sharded handle is driven stage by stage");
    HIPCHK(hipSetDevice(h->device));
    int rc = ensure_async(h);
    if (rc != TSLAM_OK) return rc;
    const int k = (int)(h->as_batches & 1);
    if (h->as_staged_armed[k]) {
        HIPCHK(hipEventSynchronize(h->as_staged[k]));
        h->as_staged_armed[k] = false;
    }
    *stage = (uint8_t*)h->as_stage[k];
    if (frame_bytes) *frame_bytes = host_frame_bytes(h);
    return TSLAM_OK;
}

int tslam_submit_host(tslam_handle* h, const uint8_t* host_images, const double* timestamps, int n_frames) {
    if (!h || !host_images) return fail(TSLAM_EINVAL, "bad argument");
    if (n_frames < 1 || n_frames > h->B) return fail(TSLAM_EINVAL, "n_frames must be in [1, max_batch]");
    if (h->sh_world > 1 || h->sh_comm) return fail(TSLAM_ESTATE, "a sharded handle is driven stage by stage");
    HIPCHK(hipSetDevice(h->device));
    int rc = ensure_async(h);
    if (rc != TSLAM_OK) return rc;
    const int k = (int)(h->as_batches & 1);
    const size_t bytes = (size_t)n_frames * host_frame_bytes(h);
    // the staging buffer of this parity is free once the DMA of batch s-2 out of it finished
    if (h->as_staged_armed[k]) HIPCHK(hipEventSynchronize(h->as_staged[k]));
    if (host_images != h->as_stage[k]) memcpy(h->as_stage[k], host_images, bytes);   // (tslam_host_stage: in place)
    // the device input of this parity: batch s-2's rectify read it earlier on the same stream
    HIPCHK(hipMemcpyAsync(h->as_input[k], h->as_stage[k], bytes, hipMemcpyHostToDevice, h->as_front));
    HIPCHK(hipEventRecord(h->as_staged[k], h->as_front));
    h->as_staged_armed[k] = true;
    if ((rc = tslam_begin_batch(h, h->as_input[k], n_frames)) != TSLAM_OK) return rc;
    const int stages[5] = {TSLAM_STAGE_RECTIFY, TSLAM_STAGE_DETECT, TSLAM_STAGE_DESCRIBE, TSLAM_STAGE_MATCH, TSLAM_STAGE_POSE};
    for (int i = 0; i < 5 && rc == TSLAM_OK; ++i) rc = tslam_run_stage(h, stages[i], i < 3 ? h->as_front : h->as_back);
    // results of this batch into the pinned slot of its parity, copied on the back stream right
    // after its pose stage: the next batch's back stages overwrite the pose buffers in that
    // stream's order, so the copies read this batch's records whatever the BA stream does
    if (rc == TSLAM_OK) rc = stash_results(h, timestamps, h->as_back);
    if (rc == TSLAM_OK && h->prm.ba_window) {
        // the BA stream waits for the back stream (ba_stage's event is recorded after the copies),
        // and the slot is ready once this batch's BA ran: the caller reads the window after polling
        rc = tslam_run_stage(h, TSLAM_STAGE_BA, h->as_ba);
        BA_FLUSH(h);   // the slot event below follows the BA's launches
        if (rc == TSLAM_OK) HIPCHK(hipEventRecord(h->as_res[(h->as_batches - 1) & 1].ev, h->as_ba));
    }
    const int rc2 = tslam_end_batch(h);
    return rc != TSLAM_OK ? rc : rc2;
}

static void unpack_records(const double* pose, int n, double* T_rel, double* T_abs, double* cov) {
    for (int i = 0; i < n; ++i) {
        const double* src = pose + (size_t)i * TS_POSE_DOUBLES;
        if (T_rel) memcpy(T_rel + 16 * (size_t)i, src, 16 * sizeof(double));
        if (T_abs) memcpy(T_abs + 16 * (size_t)i, src + 16, 16 * sizeof(double));
        if (cov) memcpy(cov + 36 * (size_t)i, src + 32, 36 * sizeof(double));
    }
}

int tslam_poll_batch(tslam_handle* h, int block, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats,
                     double* rig_T_rel, double* rig_T_abs, double* rig_cov, int32_t* rig_stats, double* ts,
                     int64_t* first_frame, int* n_frames) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    HIPCHK(hipSetDevice(h->device));
    // the oldest unread batch
    int k = -1;
    for (int i = 0; i < 2; ++i)
        if (h->as_res[i].pending && (k < 0 || h->as_res[i].batch < h->as_res[k].batch)) k = i;
    if (k < 0) return 0;
    auto& r = h->as_res[k];
    if (block) {
        HIPCHK(hipEventSynchronize(r.ev));
    } else {
        const hipError_t q = hipEventQuery(r.ev);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return fail(TSLAM_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    if (max_frames < r.n) return fail(TSLAM_EINVAL, "output capacity (max_frames) is smaller than the batch");
    const int np = r.n * h->P;
    unpack_records(r.pose, np, T_rel, T_abs, cov);
    if (stats) memcpy(stats, r.stats, sizeof(int32_t) * TS_STATS_INTS * np);
    if (h->rig) {
        unpack_records(r.rig_pose, r.n, rig_T_rel, rig_T_abs, rig_cov);
        if (rig_stats) memcpy(rig_stats, r.rig_stats, sizeof(int32_t) * TS_STATS_INTS * r.n);
    }
    if (ts) memcpy(ts, r.ts.data(), sizeof(double) * r.n);
    if (first_frame) *first_frame = r.g0;
    if (n_frames) *n_frames = r.n;
    r.pending = false;
    return 1;
}

int tslam_poll_pose(tslam_handle* h, double* T, double* cov, double* ts, int32_t* state, float* conf) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    HIPCHK(hipSetDevice(h->device));
    int k = -1;   // the newest completed batch
    for (int i = 0; i < 2; ++i) {
        const auto& r = h->as_res[i];
        if (r.batch < 0 || r.batch <= h->as_last_pose_batch || (k >= 0 && r.batch < h->as_res[k].batch)) continue;
        const hipError_t q = hipEventQuery(r.ev);
        if (q == hipErrorNotReady) continue;
        if (q != hipSuccess) return fail(TSLAM_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
        k = i;
    }
    if (k < 0) return 0;
    const auto& r = h->as_res[k];
    const int f = r.n - 1;
    const double* rec = h->rig ? r.rig_pose + (size_t)f * TS_POSE_DOUBLES : r.pose + (size_t)f * h->P * TS_POSE_DOUBLES;
    const int32_t* st = h->rig ? r.rig_stats + (size_t)f * TS_STATS_INTS : r.stats + (size_t)f * h->P * TS_STATS_INTS;
    if (T) memcpy(T, rec + 16, 16 * sizeof(double));
    if (cov) memcpy(cov, rec + 32, 36 * sizeof(double));
    if (ts) *ts = r.ts[f];
    if (state) *state = st[0];
    if (conf) {   // isaac_ros.py:312: clamp(1 / (1 + trace(cov[:3, :3])), 0, 1); 1 when not tracked
        const double tr = rec[32] + rec[32 + 7] + rec[32 + 14];
        *conf = st[0] == TSLAM_POSE_OK ? (float)std::min(1.0, std::max(0.0, 1.0 / (1.0 + tr))) : 1.0f;
    }
    h->as_last_pose_batch = r.batch;
    return 1;
}

int64_t tslam_frames_done(tslam_handle* h) { return h ? h->frames_done : -1; }

int tslam_begin_batch(tslam_handle* h, const uint8_t* images, int n_frames) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!images) return fail(TSLAM_EINVAL, "null images");
    if (n_frames < 1 || n_frames > h->B) return fail(TSLAM_EINVAL, "n_frames must be in [1, max_batch]");
    if (h->in_batch) return fail(TSLAM_ESTATE, "previous batch not ended");
    h->cur_images = images;
    h->cur_n = n_frames;
    h->cur_g0 = h->frames_done;
    h->in_batch = true;
    h->batch_started = false;
    h->front_started = h->back_started = false;
    h->front_stream = h->back_stream = nullptr;
    return TSLAM_OK;
}

int tslam_end_batch(tslam_handle* h) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "no batch in progress");
    h->frames_done += h->cur_n;
    h->in_batch = false;
    if (h->prior_armed) {   // the prior slot of this parity is free once this batch's last stage ran
        const int par = (int)(h->batch_idx & 1);
        if (!h->ev_prior[par]) HIPCHK(hipEventCreateWithFlags(&h->ev_prior[par], hipEventDisableTiming));
        HIPCHK(hipEventRecord(h->ev_prior[par], h->last_stream));
        h->prior_read_armed[par] = true;
    }
    h->prior_armed = false;   // a prior applies to one batch
    h->prior_copy_pending = false;
    if (h->back_started && h->front_started && h->back_stream != h->front_stream) {
        const int par = (int)(h->batch_idx & 1);
        HIPCHK(hipEventRecord(h->ev_back[par], h->back_stream));
        h->back_pending[par] = true;
    }
    h->batch_idx += 1;
    return TSLAM_OK;
}

// tslam_loop_auto: the batch's keyframes into the database, right after its pose stage
static void loop_auto_store(tslam_handle* h, const BatchCtx& c, hipStream_t s) {
    if (!h->lp_auto) return;
    const LoopDb db{h->d_lp_xyz, h->d_lp_desc, h->d_lp_n, h->d_lp_snap_kps, h->d_lp_snap_kcount, h->d_lp_snap_desc};
    launch_loop_store_auto(c, h->lp_auto, db, h->lp_cap / h->P, h->rig, h->d_lp_pos, s);
    if (hipEventRecord(h->lp_ev_store, s) == hipSuccess) h->lp_store_armed = true;
}

int tslam_run_stage(tslam_handle* h, int stage, void* stream) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "tslam_begin_batch first");
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const bool front = stage == TSLAM_STAGE_ALL || stage == TSLAM_STAGE_RECTIFY || stage == TSLAM_STAGE_DETECT ||
                       stage == TSLAM_STAGE_DESCRIBE || (stage >= TSLAM_KERNEL_RECTIFY_PYRAMID && stage <= TSLAM_KERNEL_DESCRIBE);
    const bool back = stage == TSLAM_STAGE_ALL || stage == TSLAM_STAGE_MATCH || stage == TSLAM_STAGE_POSE ||
                      (stage >= TSLAM_KERNEL_MATCH && stage <= TSLAM_KERNEL_POSE_SOLVE);
    if (!h->ev_front) {
        HIPCHK(hipEventCreateWithFlags(&h->ev_front, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_back[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_back[1], hipEventDisableTiming));
    }
    const int par = (int)(h->batch_idx & 1);
    if (back && !h->back_started) BA_FLUSH(h);   // a deferred BA of the previous batch: now, behind this batch's front
    if (stage != TSLAM_STAGE_BA && !h->batch_started) {
        if (h->ba_job.pending && h->ba_job.par == par) ba_flush(h);   // (that BA's event is recorded before this wait)
        // the first work of a batch: the BA of the batch two back (same ring slots) must be done
        if (h->ba_pending[par]) HIPCHK(hipStreamWaitEvent(s, h->ev_ba[par], 0));
        h->ba_pending[par] = false;
        h->batch_started = true;
    }
    if (front && !h->front_started) {
        // ... and so must the back stages of the batch two back (they read the frames whose ring
        // slots this batch's front stages overwrite)
        if (h->back_pending[par]) HIPCHK(hipStreamWaitEvent(s, h->ev_back[par], 0));
        h->back_pending[par] = false;
        h->front_started = true;
        h->front_stream = s;
    }
    if (back && !h->back_started) {
        if (h->front_started && h->front_stream != s) {   // this batch's features come from the front stream
            HIPCHK(hipEventRecord(h->ev_front, h->front_stream));
            HIPCHK(hipStreamWaitEvent(s, h->ev_front, 0));
        }
        h->back_started = true;
        h->back_stream = s;
    }
    if (back && h->prior_copy_pending) {   // this batch's prior (tslam_set_motion_prior), before its pose stage
        const size_t slot = (size_t)TS_PRIOR_DOUBLES * h->P * h->B;
        HIPCHK(hipMemcpyAsync(h->d_prior + (size_t)par * slot, h->h_prior_pin[par], sizeof(double) * slot,
                              hipMemcpyHostToDevice, s));
        h->prior_copy_pending = false;
    }
    if (front && h->front_started && s != h->front_stream && !back)
        return fail(TSLAM_ESTATE, "all front stages of a batch must use one stream");
    if (back && h->back_started && s != h->back_stream && !front)
        return fail(TSLAM_ESTATE, "all back stages of a batch must use one stream");
    if (stage != TSLAM_STAGE_BA) h->last_stream = s;
    const BatchCtx c = make_ctx(h);
    if (h->sh_world > 1 || h->sh_comm) return run_sharded_stage(h, c, stage, s);
    if (h->prm.rgbd && (stage == TSLAM_STAGE_RECTIFY || stage == TSLAM_STAGE_ALL || stage == TSLAM_KERNEL_RECTIFY_PYRAMID))
        launch_rgbd_gray(c, h->d_gray, s);   // the colour images become the gray input of rectify
    switch (stage) {
        case TSLAM_STAGE_RECTIFY: launch_rectify_pyramid(c, s); break;
        case TSLAM_STAGE_DETECT: launch_detect(c, s); launch_select(c, s); break;
        case TSLAM_STAGE_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_STAGE_MATCH: launch_match(c, s); launch_match_refine(c, s); break;
        case TSLAM_STAGE_POSE:
            launch_pose(c, s);
            if (h->rig) launch_rig_pose(c, s);
            launch_chains(c, h->rig, s);
            loop_auto_store(h, c, s);
            break;
        case TSLAM_STAGE_ALL:
            launch_rectify_pyramid(c, s);
            launch_detect(c, s);
            launch_select(c, s);
            launch_describe(c, s);
            launch_match(c, s);
            launch_match_refine(c, s);
            launch_pose(c, s);
            if (h->rig) launch_rig_pose(c, s);
            launch_chains(c, h->rig, s);
            loop_auto_store(h, c, s);
            if (h->prm.ba_window) {
                double* snap = h->ba.fe_pose + (size_t)(h->batch_idx & 1) * h->B * h->P * 16;
                double* snap_body = h->ba.fe_body + (size_t)(h->batch_idx & 1) * h->B * 16;
                int32_t* assoc = h->ba.kf_assoc + (size_t)(h->batch_idx & 1) * h->B * h->P * h->g.K;
                launch_ba_snapshot(c, snap, s);
                launch_ba_kf_assoc(c, assoc, h->prm.ba_kf_interval, s);
                if (ba_rig(h)) launch_ba_snapshot_rig(c, snap_body, s);
                if (const hipError_t e = run_ba(h, c, s, snap, snap_body, assoc); e != hipSuccess)
                    return fail(TSLAM_EHIP, std::string("BA: ") + hipGetErrorString(e));
            }
            break;
        case TSLAM_KERNEL_RIG:
            if (!h->rig) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
            launch_rig_pose(c, s);
            break;
        case TSLAM_STAGE_BA: {
            const int rc = ba_stage(h, c, s);
            if (rc != TSLAM_OK) return rc;
            break;
        }
        case TSLAM_KERNEL_RECTIFY_PYRAMID: launch_rectify_pyramid(c, s); break;
        case TSLAM_KERNEL_DETECT: launch_detect(c, s); break;
        case TSLAM_KERNEL_SELECT: launch_select(c, s); break;
        case TSLAM_KERNEL_DESCRIBE: launch_describe(c, s); break;
        case TSLAM_KERNEL_MATCH: launch_match(c, s); break;
        case TSLAM_KERNEL_MATCH_REFINE: launch_match_refine(c, s); break;
        case TSLAM_KERNEL_POSE: launch_pose(c, s); break;
        case TSLAM_KERNEL_POSE_SOLVE: launch_pose_solve(c, s); break;
        case TSLAM_KERNEL_CHAIN: launch_chains(c, h->rig, s); break;
        default: return fail(TSLAM_EINVAL, "unknown stage");
    }
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_submit(tslam_handle* h, const uint8_t* images, int n_frames, void* stream) {
    int rc = tslam_begin_batch(h, images, n_frames);
    if (rc != TSLAM_OK) return rc;
    rc = tslam_run_stage(h, TSLAM_STAGE_ALL, stream);
    const int rc2 = tslam_end_batch(h);
    return rc != TSLAM_OK ? rc : rc2;
}

int tslam_detect(tslam_handle* h, void* stream) {
    int rc = tslam_run_stage(h, TSLAM_STAGE_RECTIFY, stream);
    return rc != TSLAM_OK ? rc : tslam_run_stage(h, TSLAM_STAGE_DETECT, stream);
}
int tslam_describe(tslam_handle* h, void* stream) { return tslam_run_stage(h, TSLAM_STAGE_DESCRIBE, stream); }
int tslam_match(tslam_handle* h, void* stream) { return tslam_run_stage(h, TSLAM_STAGE_MATCH, stream); }
int tslam_pose(tslam_handle* h, void* stream) { return tslam_run_stage(h, TSLAM_STAGE_POSE, stream); }

int tslam_sync(tslam_handle* h) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    return TSLAM_OK;
}

static int copy_pose_records(const double* dev_pose, const int32_t* dev_stats, int n, double* T_rel, double* T_abs,
                             double* cov, int32_t* stats) {
    std::vector<double> pose((size_t)n * TS_POSE_DOUBLES);
    HIPCHK(hipMemcpy(pose.data(), dev_pose, sizeof(double) * pose.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        const double* src = pose.data() + (size_t)i * TS_POSE_DOUBLES;
        if (T_rel) memcpy(T_rel + 16 * (size_t)i, src, 16 * sizeof(double));
        if (T_abs) memcpy(T_abs + 16 * (size_t)i, src + 16, 16 * sizeof(double));
        if (cov) memcpy(cov + 36 * (size_t)i, src + 32, 36 * sizeof(double));
    }
    if (stats) HIPCHK(hipMemcpy(stats, dev_stats, sizeof(int32_t) * TS_STATS_INTS * (size_t)n, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_read_poses(tslam_handle* h, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (h->cur_n == 0) return fail(TSLAM_ESTATE, "no batch has run since tslam_create / tslam_reset");
    if (max_frames < h->cur_n) return fail(TSLAM_EINVAL, "output capacity (max_frames) is smaller than the last batch");
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    return copy_pose_records((const double*)h->buf[TSLAM_BUF_POSE].ptr, (const int32_t*)h->buf[TSLAM_BUF_STATS].ptr,
                             h->cur_n * h->P, T_rel, T_abs, cov, stats);
}

int tslam_buffer_info(tslam_handle* h, int which, void** device_ptr, int64_t* bytes_total, int64_t* bytes_per_frame) {
    if (!h || which < 0 || which >= TSLAM_BUF_COUNT) return fail(TSLAM_EINVAL, "bad handle or buffer id");
    BA_FLUSH(h);
    if (device_ptr) *device_ptr = h->buf[which].ptr;
    if (bytes_total) *bytes_total = h->buf[which].bytes;
    if (bytes_per_frame) *bytes_per_frame = h->buf[which].per_frame;
    return TSLAM_OK;
}

int tslam_copy_out(tslam_handle* h, int which, int64_t offset, void* host_dst, int64_t bytes) {
    if (!h || which < 0 || which >= TSLAM_BUF_COUNT || !host_dst) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (offset < 0 || bytes < 0 || offset + bytes > h->buf[which].bytes) return fail(TSLAM_EINVAL, "range outside buffer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(host_dst, (const char*)h->buf[which].ptr + offset, (size_t)bytes, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_copy_in(tslam_handle* h, int which, int64_t offset, const void* host_src, int64_t bytes) {
    if (!h || which < 0 || which >= TSLAM_BUF_COUNT || !host_src) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (offset < 0 || bytes < 0 || offset + bytes > h->buf[which].bytes) return fail(TSLAM_EINVAL, "range outside buffer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy((char*)h->buf[which].ptr + offset, host_src, (size_t)bytes, hipMemcpyHostToDevice));
    return TSLAM_OK;
}

int tslam_ring_slot(tslam_handle* h, int64_t global_frame) {
    if (!h || global_frame < 0) return fail(TSLAM_EINVAL, "bad argument");
    return (int)(global_frame % h->R);
}

int tslam_layout(tslam_handle* h, int64_t* out16, int32_t* level_info18) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (out16) {
        for (int i = 0; i < 16; ++i) out16[i] = 0;
        out16[0] = h->W;
        out16[1] = h->H;
        out16[2] = h->g.n_levels;
        out16[3] = h->g.K;
        out16[4] = h->R;
        out16[5] = h->B;
        out16[6] = h->P;
        out16[7] = h->g.pyr_bytes;
        for (int l = 0; l < h->g.n_levels; ++l) out16[8 + l] = h->g.pyr_off[l];
    }
    if (level_info18) {
        for (int i = 0; i < 18; ++i) level_info18[i] = 0;
        for (int l = 0; l < h->g.n_levels; ++l) {
            level_info18[3 * l] = h->g.W[l];
            level_info18[3 * l + 1] = h->g.H[l];
            level_info18[3 * l + 2] = h->g.Kq[l];
        }
    }
    return TSLAM_OK;
}

int tslam_set_motion_prior(tslam_handle* h, const double* prior, int n_frames) {
    if (!h || !prior) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_set_motion_prior inside a batch");
    if (n_frames < 1 || n_frames > h->B) return fail(TSLAM_EINVAL, "n_frames must be in [1, max_batch]");
    HIPCHK(hipSetDevice(h->device));
    const size_t slot = (size_t)TS_PRIOR_DOUBLES * h->P * h->B;
    if (!h->d_prior) {   // one slot per batch parity: batch s-1 may still be reading its prior
        const int rc = dev_alloc(h, (void**)&h->d_prior, sizeof(double) * 2 * slot);
        if (rc != TSLAM_OK) return rc;
    }
    if (h->rig && !h->d_rig_prior) {
        const int rc = dev_alloc(h, (void**)&h->d_rig_prior, sizeof(double) * 2 * TS_PRIOR_DOUBLES * h->B);
        if (rc != TSLAM_OK) return rc;
    }
    // the slot's previous reader is batch s-2 (pose + chain stages): wait for the event its last
    // stage recorded, not for the whole device
    const int par = (int)(h->batch_idx & 1);
    if (h->prior_read_armed[par]) {
        HIPCHK(hipEventSynchronize(h->ev_prior[par]));
        h->prior_read_armed[par] = false;
    }
    if (!h->h_prior_pin[par]) {
        HIPCHK(hipHostMalloc((void**)&h->h_prior_pin[par], sizeof(double) * slot, hipHostMallocDefault));
        h->host_allocs.push_back(h->h_prior_pin[par]);
    }
    // pinned staging (its previous DMA, batch s-2's, is covered by the event above); the copy is
    // enqueued on the batch's own back stream, so no host wait and no null-stream ordering
    const size_t nb = (size_t)TS_PRIOR_DOUBLES * h->P * n_frames;
    memcpy(h->h_prior_pin[par], prior, sizeof(double) * nb);
    std::fill(h->h_prior_pin[par] + nb, h->h_prior_pin[par] + slot, 0.0);   // frames past n: weight 0
    h->prior_armed = true;
    h->prior_copy_pending = true;
    return TSLAM_OK;
}

static int set_rig_E(tslam_handle* h, int q_total, const double* base_T_rect) {
    HIPCHK(hipSetDevice(h->device));
    std::vector<double> e(32 * (size_t)q_total, 0.0);
    for (int q = 0; q < q_total; ++q) {
        const double* E = base_T_rect + 16 * q;
        double* inv = e.data() + 16 * (q_total + q);
        for (int i = 0; i < 16; ++i) e[16 * q + i] = E[i];
        if (E[12] != 0.0 || E[13] != 0.0 || E[14] != 0.0 || E[15] != 1.0) return fail(TSLAM_EINVAL, "base_T_rect must be rigid 4x4");
        for (int i = 0; i < 3; ++i) {   // [R^T | -R^T t]
            for (int j = 0; j < 3; ++j) inv[4 * i + j] = E[4 * j + i];
            inv[4 * i + 3] = -((E[i] * E[3] + E[4 + i] * E[7]) + E[8 + i] * E[11]);
        }
        inv[15] = 1.0;
    }
    if (q_total > h->rig_cap) {
        if (h->d_rig_E) {
            (void)hipFree(h->d_rig_E);
            h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), (void*)h->d_rig_E), h->allocs.end());
            h->d_rig_E = nullptr;
        }
        const int rc = dev_alloc(h, (void**)&h->d_rig_E, sizeof(double) * 32 * q_total);
        if (rc != TSLAM_OK) return rc;
        h->rig_cap = q_total;
    }
    if (!h->d_rig_pose) {
        int rc = dev_alloc(h, (void**)&h->d_rig_pose, sizeof(double) * TS_POSE_DOUBLES * h->B);
        if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rig_stats, sizeof(int32_t) * TS_STATS_INTS * h->B);
        if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rig_state, sizeof(double) * 32);   // chain (A, Q)
        if (rc != TSLAM_OK) return rc;
        const double eye[32] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        HIPCHK(hipMemcpy(h->d_rig_state, eye, sizeof(eye), hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemcpy(h->d_rig_E, e.data(), sizeof(double) * e.size(), hipMemcpyHostToDevice));
    h->rig_q = q_total;
    return TSLAM_OK;
}

int tslam_set_rig(tslam_handle* h, const double* base_T_rect) {
    if (!h || !base_T_rect) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_set_rig inside a batch");
    const int rc = set_rig_E(h, h->P, base_T_rect);
    if (rc != TSLAM_OK) return rc;
    h->rig = true;
    return TSLAM_OK;
}

int tslam_read_rig_poses(tslam_handle* h, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (!h->rig) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
    if (h->cur_n == 0) return fail(TSLAM_ESTATE, "no batch has run since tslam_create / tslam_reset");
    if (max_frames < h->cur_n) return fail(TSLAM_EINVAL, "output capacity (max_frames) is smaller than the last batch");
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    return copy_pose_records(h->d_rig_pose, h->d_rig_stats, h->cur_n, T_rel, T_abs, cov, stats);
}

// -- sharded rig ------------------------------------------------------------------
int tslam_set_shard(tslam_handle* h, int cam_lo, int cam_hi, int rank, int world) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_set_shard inside a batch");
    if (cam_lo < 0 || cam_hi > h->C || cam_lo >= cam_hi) return fail(TSLAM_EINVAL, "camera range outside [0, cameras)");
    if (world < 1 || rank < 0 || rank >= world || world > h->B) return fail(TSLAM_EINVAL, "need 0 <= rank < world <= max_batch");
    if (world > 1 && h->prm.ba_window && h->prm.rgbd)
        return fail(TSLAM_EINVAL, "a camera-sharded RGB-D rig runs without local BA");
    h->sh_cam_lo = cam_lo;
    h->sh_cam_hi = cam_hi;
    h->sh_rank = rank;
    h->sh_world = world;
    h->sh_pairs = false;   // the driver sets the pair split after (tslam_shard_options)
    return TSLAM_OK;
}

int tslam_exchange_sizes(tslam_handle* h, int64_t* stream_block, int64_t* pose_record) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (stream_block) *stream_block = stream_block_bytes(h->g);
    if (pose_record) *pose_record = pose_record_bytes(h->P);
    return TSLAM_OK;
}

static int check_frames_cams(tslam_handle* h, int64_t first_frame, int n_frames, int cam_lo, int cam_hi) {
    if (n_frames < 1 || n_frames > h->R) return fail(TSLAM_EINVAL, "n_frames must be in [1, ring]");
    if (cam_lo < 0 || cam_hi > h->C || cam_lo >= cam_hi) return fail(TSLAM_EINVAL, "camera range outside [0, cameras)");
    if (first_frame + n_frames < 0) return fail(TSLAM_EINVAL, "frame range before the sequence start");
    return TSLAM_OK;
}

int tslam_pack_streams(tslam_handle* h, int64_t first_frame, int n_frames, int cam_lo, int cam_hi, void* dst, void* stream) {
    if (!h || !dst) return fail(TSLAM_EINVAL, "bad argument");
    int rc = check_frames_cams(h, first_frame, n_frames, cam_lo, cam_hi);
    if (rc != TSLAM_OK) return rc;
    HIPCHK(hipSetDevice(h->device));
    launch_stream_blocks(make_ctx(h), true, first_frame, n_frames, cam_lo, cam_hi - cam_lo, (uint8_t*)dst, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_unpack_streams(tslam_handle* h, int64_t first_frame, int n_frames, int cam_lo, int cam_hi, const void* src,
                         void* stream) {
    if (!h || !src) return fail(TSLAM_EINVAL, "bad argument");
    int rc = check_frames_cams(h, first_frame, n_frames, cam_lo, cam_hi);
    if (rc != TSLAM_OK) return rc;
    HIPCHK(hipSetDevice(h->device));
    launch_stream_blocks(make_ctx(h), false, first_frame, n_frames, cam_lo, cam_hi - cam_lo, (uint8_t*)src, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_import_raw(tslam_handle* h, const uint8_t* images, int64_t first_frame, int n_frames, int cam_lo, int cam_hi,
                     void* stream) {
    if (!h || !images) return fail(TSLAM_EINVAL, "bad argument");
    int rc = check_frames_cams(h, first_frame, n_frames, cam_lo, cam_hi);
    if (rc != TSLAM_OK) return rc;
    if (h->prm.rgbd) return fail(TSLAM_EINVAL, "tslam_import_raw takes gray stereo images");
    HIPCHK(hipSetDevice(h->device));
    BatchCtx c = make_ctx(h);
    const int ncam = cam_hi - cam_lo;
    const int64_t skip = first_frame < 0 ? -first_frame : 0;   // frames before the sequence start
    c.images = images + (size_t)skip * ncam * h->W * h->H;
    c.g0 = first_frame + skip;
    c.n = (int)(n_frames - skip);
    c.cam0 = cam_lo;
    c.ncam = ncam;
    launch_rectify_pyramid(c, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_pair_block_bytes(tslam_handle* h, int64_t* bytes) {
    if (!h || !bytes) return fail(TSLAM_EINVAL, "bad argument");
    *bytes = pair_block_bytes(h->g);
    return TSLAM_OK;
}

static int pair_blocks(tslam_handle* h, bool pack, int f0, int n_frames, int pair_lo, int pair_hi, uint8_t* buf, void* stream) {
    if (!h || !buf) return fail(TSLAM_EINVAL, "bad argument");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "pair blocks are packed / unpacked inside a batch");
    if (f0 < 0 || n_frames < 1 || f0 + n_frames > h->cur_n) return fail(TSLAM_EINVAL, "frame range outside the batch");
    if (pair_lo < 0 || pair_hi > h->P || pair_lo >= pair_hi) return fail(TSLAM_EINVAL, "pair range outside [0, pairs)");
    HIPCHK(hipSetDevice(h->device));
    launch_pair_blocks(make_ctx(h), pack, f0, n_frames, pair_lo, pair_hi - pair_lo, buf, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_pack_pairs(tslam_handle* h, int f0, int n_frames, int pair_lo, int pair_hi, void* dst, void* stream) {
    return pair_blocks(h, true, f0, n_frames, pair_lo, pair_hi, (uint8_t*)dst, stream);
}

int tslam_unpack_pairs(tslam_handle* h, int f0, int n_frames, int pair_lo, int pair_hi, const void* src, void* stream) {
    return pair_blocks(h, false, f0, n_frames, pair_lo, pair_hi, (uint8_t*)src, stream);
}

int tslam_internal_info(tslam_handle* h, tslam_handle_info* o) {
    if (!h || !o) return fail(TSLAM_EINVAL, "bad argument");
    o->device = h->device;
    o->W = h->W;
    o->H = h->H;
    o->P = h->P;
    o->C = h->C;
    o->B = h->B;
    o->rgbd = h->prm.rgbd;
    o->rig = h->rig ? 1 : 0;
    o->ba = h->prm.ba_window;
    o->frames_done = h->frames_done;
    o->stream_block = stream_block_bytes(h->g);
    o->pose_record = pose_record_bytes(h->P);
    o->pair_block = pair_block_bytes(h->g);
    o->cam_lo = h->sh_cam_lo;
    o->cam_hi = h->sh_cam_hi;
    o->rank = h->sh_rank;
    o->world = h->sh_world;
    return TSLAM_OK;
}

int tslam_internal_attach_driver(tslam_handle* h, tslam_shard_driver* d, bool owned) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (h->drv && h->drv_owned && h->drv != d) tslam_internal_driver_destroy(h->drv);
    h->drv = d;
    h->drv_owned = d && owned;
    h->sh_comm = d != nullptr;
    return TSLAM_OK;
}

tslam_shard_driver* tslam_internal_driver(tslam_handle* h) { return h ? h->drv : nullptr; }

int64_t tslam_internal_state_bytes(tslam_handle* h, int n, int rank, int cam_lo, int cam_hi) {
    int lo, hi;
    peer_range(rank, n, h->sh_world, &lo, &hi);
    const int left0 = (cam_lo + 1) & ~1, nleft = cam_hi > left0 ? (cam_hi - left0 + 1) / 2 : 0;
    return (int64_t)(hi - lo) * h->P * state_range_block_bytes(h->g) + (int64_t)n * nleft * state_camera_block_bytes(h->g);
}

int tslam_internal_state_blocks(tslam_handle* h, int pack, int rank, int cam_lo, int cam_hi, void* buf, void* stream) {
    if (!h || !buf) return fail(TSLAM_EINVAL, "bad argument");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "state blocks are packed / unpacked inside a batch");
    if (h->prm.rgbd) return fail(TSLAM_ESTATE, "state blocks describe a stereo rig");
    HIPCHK(hipSetDevice(h->device));
    launch_state_blocks(make_ctx(h), pack != 0, h->cur_n, h->sh_world, rank, cam_lo, cam_hi, (uint8_t*)buf,
                        (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_perturb_temporal(tslam_handle* h, int percent, uint64_t seed, void* stream) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (!h->in_batch) return fail(TSLAM_ESTATE, "tslam_perturb_temporal inside a batch (after MATCH_REFINE)");
    if (percent < 0 || percent > 100) return fail(TSLAM_EINVAL, "percent must be in [0, 100]");
    if (h->sh_world > 1 || h->sh_comm) return fail(TSLAM_ESTATE, "tslam_perturb_temporal takes an unsharded handle");
    HIPCHK(hipSetDevice(h->device));
    if (percent > 0) launch_perturb_uv(make_ctx(h), percent, seed, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_internal_stash(tslam_handle* h, void* stream) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "results are stashed inside a batch (before tslam_end_batch)");
    HIPCHK(hipSetDevice(h->device));
    return stash_results(h, nullptr, (hipStream_t)stream);
}

// -- the all-to-all's peers in one launch each (alltoall layout [world][nr][S]) -------------------
static int check_peers(tslam_handle* h) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "peer exchange blocks are packed / imported inside a batch");
    if (h->sh_world < 2 || h->prm.rgbd) return fail(TSLAM_ESTATE, "a stereo handle sharded over world > 1");
    if ((h->sh_cam_hi - h->sh_cam_lo) * h->sh_world != h->C || h->sh_cam_lo != h->sh_rank * (h->sh_cam_hi - h->sh_cam_lo))
        return fail(TSLAM_EINVAL, "peer layout needs cameras [rank*S, (rank+1)*S)");
    return TSLAM_OK;
}

int tslam_pack_streams_peers(tslam_handle* h, void* dst, void* stream) {
    int rc = check_peers(h);
    if (rc != TSLAM_OK) return rc;
    if (!dst) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    const int N = h->sh_world, S = h->sh_cam_hi - h->sh_cam_lo;
    launch_stream_blocks_peers(make_ctx(h), true, h->cur_g0, h->cur_n, N, peer_cap(h->B, N), h->sh_rank, S, (uint8_t*)dst,
                               (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_stage_raw_peers(tslam_handle* h, const uint8_t* prev_raw, void* dst, void* stream) {
    int rc = check_peers(h);
    if (rc != TSLAM_OK) return rc;
    if (!prev_raw || !dst) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    const int N = h->sh_world, S = h->sh_cam_hi - h->sh_cam_lo;
    launch_stage_raw_peers(h->cur_images, prev_raw, (uint8_t*)dst, h->cur_n, N, peer_cap(h->B, N), h->sh_rank, S,
                           (int64_t)h->W * h->H, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_import_peers(tslam_handle* h, const uint8_t* raw, const void* streams, void* stream) {
    int rc = check_peers(h);
    if (rc != TSLAM_OK) return rc;
    if (!raw || !streams) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    const int N = h->sh_world, S = h->sh_cam_hi - h->sh_cam_lo, cap = peer_cap(h->B, N);
    const int nr = peer_frames(h->sh_rank, h->cur_n, N);
    if (nr == 0) return TSLAM_OK;   // an empty frame range: this rank's back end has nothing to do
    int lo, hi;
    shard_range(h, h->cur_n, &lo, &hi);
    const int64_t first = h->cur_g0 + lo - 1;
    const int skip = first < 0 ? 1 : 0;   // frame -1 (before the sequence start) is not imported
    BatchCtx c = make_ctx(h);
    c.images = raw;
    c.g0 = first + skip;
    c.n = nr - skip;
    c.peer_S = S;
    c.peer_me = h->sh_rank;
    c.peer_nbuf = cap;
    c.peer_skip = skip;
    if (c.n > 0) launch_rectify_pyramid(c, (hipStream_t)stream);
    launch_stream_blocks_peers(make_ctx(h), false, h->cur_g0, h->cur_n, N, cap, h->sh_rank, S, (uint8_t*)streams,
                               (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

// -- pair split (TSLAM_SHARD_PAIRS): the partner camera's frames of this rank's half -------------
int tslam_internal_set_pairs(tslam_handle* h, int on) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (h->in_batch) return fail(TSLAM_ESTATE, "the pair split is set outside a batch");
    if (on) {
        if (h->prm.rgbd) return fail(TSLAM_EINVAL, "the pair split shards a stereo rig");
        if (h->sh_world < 2 || h->sh_world != h->C || h->sh_cam_hi - h->sh_cam_lo != 1 || h->sh_cam_lo != h->sh_rank)
            return fail(TSLAM_EINVAL, "the pair split needs one camera per rank (world = cameras)");
        if (h->prm.ba_window) return fail(TSLAM_EINVAL, "the pair split runs without local BA (no state gather)");
    }
    h->sh_pairs = on != 0;
    return TSLAM_OK;
}

static int check_partner(tslam_handle* h) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "partner blocks are packed / imported inside a batch");
    if (!h->sh_pairs) return fail(TSLAM_ESTATE, "the handle is not pair-split (TSLAM_SHARD_PAIRS)");
    return TSLAM_OK;
}

int tslam_internal_pack_partner(tslam_handle* h, void* dst, void* stream) {
    int rc = check_partner(h);
    if (rc != TSLAM_OK) return rc;
    if (!dst) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    int lo, hi;
    peer_range((h->sh_cam_lo & 1) ^ 1, h->cur_n, 2, &lo, &hi);   // the partner's half
    if (hi > lo)   // frames lo - 1 .. hi - 1 of this camera (zeros before the sequence start)
        launch_stream_blocks(make_ctx(h), true, h->cur_g0 + lo - 1, hi - lo + 1, h->sh_cam_lo, 1, (uint8_t*)dst,
                             (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_internal_import_partner(tslam_handle* h, const uint8_t* raw, const void* streams, void* stream) {
    int rc = check_partner(h);
    if (rc != TSLAM_OK) return rc;
    if (!raw || !streams) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    int lo, hi;
    pair_half(h, h->cur_n, &lo, &hi);
    if (hi <= lo) return TSLAM_OK;   // an empty half: this rank's back end has nothing to do
    const int partner = h->sh_cam_lo ^ 1, nf = hi - lo + 1;
    const int64_t first = h->cur_g0 + lo - 1;
    const int skip = first < 0 ? 1 : 0;   // frame -1 (before the sequence start) is not imported
    BatchCtx c = make_ctx(h);
    c.images = raw + (size_t)skip * h->W * h->H;
    c.g0 = first + skip;
    c.n = nf - skip;
    c.cam0 = partner;
    c.ncam = 1;
    if (c.n > 0) launch_rectify_pyramid(c, (hipStream_t)stream);
    launch_stream_blocks(make_ctx(h), false, first, nf, partner, 1, (uint8_t*)streams, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_pack_poses(tslam_handle* h, void* dst, void* stream) {
    if (!h || !dst) return fail(TSLAM_EINVAL, "bad argument");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "tslam_pack_poses inside a batch (after its POSE stage)");
    HIPCHK(hipSetDevice(h->device));
    int lo, hi;
    shard_range(h, h->cur_n, &lo, &hi);
    launch_pose_records(make_ctx(h), true, lo, hi - lo, (uint8_t*)dst, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_unpack_poses(tslam_handle* h, const void* src, void* stream) {
    if (!h || !src) return fail(TSLAM_EINVAL, "bad argument");
    if (!h->in_batch) return fail(TSLAM_ESTATE, "tslam_unpack_poses inside a batch (before its CHAIN stage)");
    HIPCHK(hipSetDevice(h->device));
    // rank q's records (its rig range) start at q * peer_records(n, world) (the all-gather pads
    // every range to the longest); with equal ranges, and no pair split, that is the batch order
    launch_pose_records_gathered(make_ctx(h), h->sh_world, h->sh_pairs, (const uint8_t*)src, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return TSLAM_OK;
}

int tslam_ba_read_map(tslam_handle* h, int pair, int64_t* gid, uint32_t* desc) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    const size_t WK = (size_t)h->prm.ba_window * h->g.K;
    if (gid) HIPCHK(hipMemcpy(gid, h->ba.gid + pair * WK, 8 * WK, hipMemcpyDeviceToHost));
    if (desc) HIPCHK(hipMemcpy(desc, h->ba.kf_desc + pair * WK * 8, 32 * WK, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

// relocalisation scratch for every pair of the handle (one pair: tslam_relocalize uses pair slot 0;
// the rig: tslam_relocalize_rig solves all pairs of one frame as a one-frame batch)
static int ensure_reloc_scratch(tslam_handle* h) {
    if (h->d_rl_match) return TSLAM_OK;
    const size_t K = h->g.K, P = h->P;
    int rc = dev_alloc(h, (void**)&h->d_rl_match, sizeof(int32_t) * K * P);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_corr, sizeof(double) * TS_CORR_DOUBLES * K * P);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_stats, sizeof(int32_t) * TS_STATS_INTS * P);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_pose, sizeof(double) * TS_POSE_DOUBLES * P);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_ransac, sizeof(uint32_t) * TS_RANSAC_WORDS * TS_MAX_SPLITS * P);
    if (rc == TSLAM_OK)
        rc = dev_alloc(h, (void**)&h->d_rl_hyp, sizeof(double) * TS_HYP_DOUBLES * 4 * (size_t)h->prm.ransac_hypotheses * P);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_rig_pose, sizeof(double) * TS_POSE_DOUBLES);
    if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_rl_rig_stats, sizeof(int32_t) * TS_STATS_INTS);
    return rc;
}

// reloc-path solve of `frame` (pair) against M landmarks; result copied to the host
// loop jobs share the relocalisation scratch and the vote buffer: the synchronous users wait for them
static int loop_quiesce(tslam_handle* h) {
    loop_worker_drain(h);
    if (h->lp_stream) HIPCHK(hipStreamSynchronize(h->lp_stream));
    return TSLAM_OK;
}

static int reloc_solve(tslam_handle* h, int pair, int64_t frame, const double* map_xyz, const uint32_t* map_desc,
                       int64_t M, double* T_out, double* cov, int32_t* stats) {
    if (loop_quiesce(h) != TSLAM_OK) return TSLAM_EHIP;
    const BatchCtx c = make_ctx(h);
    hipStream_t s = h->last_stream;
    if (M == 0) {
        const int32_t st[8] = {1, 0, 0, 0, -1, (int32_t)frame, 0, 0};
        HIPCHK(hipMemcpy(h->d_rl_stats, st, sizeof(st), hipMemcpyHostToDevice));
    } else {
        launch_reloc(c, pair, frame, map_xyz, map_desc, (int)M, h->d_rl_match, h->d_rl_corr, h->d_rl_stats,
                     h->d_rl_pose, h->d_rl_ransac, h->d_rl_hyp, s);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    double pose[TS_POSE_DOUBLES];
    HIPCHK(hipMemcpy(pose, h->d_rl_pose, sizeof(pose), hipMemcpyDeviceToHost));
    int32_t st[TS_STATS_INTS];
    HIPCHK(hipMemcpy(st, h->d_rl_stats, sizeof(st), hipMemcpyDeviceToHost));
    if (M == 0 || st[0] != 0)
        for (int i = 0; i < 16; ++i) pose[i] = (i % 5) == 0 ? 1.0 : 0.0;
    pose[12] = pose[13] = pose[14] = 0.0;   // k_refine writes the 3x4 part only
    pose[15] = 1.0;
    if (T_out) memcpy(T_out, pose, 16 * sizeof(double));
    if (cov) memcpy(cov, pose + 32, 36 * sizeof(double));
    if (stats) memcpy(stats, st, sizeof(st));
    return TSLAM_OK;
}

int tslam_map_upload(tslam_handle* h, const double* xyz, const uint32_t* desc, int64_t n) {
    if (!h || n < 0 || (n && (!xyz || !desc))) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (n > (1 << 20) - 1) return fail(TSLAM_EINVAL, "at most 2^20 - 1 map points");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    if (n > h->map_cap) {
        if (h->d_map_xyz) {   // grow: release the old buffers
            for (void* p : {(void*)h->d_map_xyz, (void*)h->d_map_desc}) {
                (void)hipFree(p);
                h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), p), h->allocs.end());
            }
        }
        int rc = dev_alloc(h, (void**)&h->d_map_xyz, sizeof(double) * 3 * n);
        if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_map_desc, sizeof(uint32_t) * 8 * n);
        if (rc != TSLAM_OK) return rc;
        h->map_cap = n;
    }
    {
        int rc = ensure_reloc_scratch(h);
        if (rc != TSLAM_OK) return rc;
    }
    if (n) {
        HIPCHK(hipMemcpy(h->d_map_xyz, xyz, sizeof(double) * 3 * n, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->d_map_desc, desc, sizeof(uint32_t) * 8 * n, hipMemcpyHostToDevice));
    }
    h->map_n = n;
    return TSLAM_OK;
}

int tslam_relocalize(tslam_handle* h, int pair, int64_t frame, double* cam_T_world, double* cov, int32_t* stats) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->d_rl_match) return fail(TSLAM_ESTATE, "no map uploaded (tslam_map_upload)");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_relocalize inside a batch");
    if (frame < 0 || frame >= h->frames_done || frame < h->frames_done - h->R)
        return fail(TSLAM_EINVAL, "frame is not resident in the ring");
    HIPCHK(hipSetDevice(h->device));
    return reloc_solve(h, pair, frame, h->d_map_xyz, h->d_map_desc, h->map_n, cam_T_world, cov, stats);
}

int tslam_relocalize_rig(tslam_handle* h, int64_t frame, double* body_T_world, double* cov, int32_t* stats,
                         int32_t* pair_stats) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (!h->rig || h->rig_q != h->P) return fail(TSLAM_ESTATE, "no rig set (tslam_set_rig)");
    if (h->prm.rgbd) return fail(TSLAM_ESTATE, "tslam_relocalize_rig takes a stereo rig");
    if (!h->d_rl_match) return fail(TSLAM_ESTATE, "no map uploaded (tslam_map_upload)");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_relocalize_rig inside a batch");
    if (frame < 0 || frame >= h->frames_done || frame < h->frames_done - h->R)
        return fail(TSLAM_EINVAL, "frame is not resident in the ring");
    HIPCHK(hipSetDevice(h->device));
    if (loop_quiesce(h) != TSLAM_OK) return TSLAM_EHIP;
    const BatchCtx c = make_ctx(h);
    hipStream_t s = h->last_stream;
    const int P = h->P;
    if (h->map_n == 0) {
        std::vector<int32_t> st(TS_STATS_INTS * (size_t)(P + 1), 0);
        for (int p = 0; p <= P; ++p) {
            st[(size_t)p * TS_STATS_INTS] = 1;
            st[(size_t)p * TS_STATS_INTS + 4] = -1;
            st[(size_t)p * TS_STATS_INTS + 5] = (int32_t)frame;
        }
        HIPCHK(hipMemcpy(h->d_rl_stats, st.data(), sizeof(int32_t) * TS_STATS_INTS * P, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->d_rl_rig_stats, st.data() + (size_t)P * TS_STATS_INTS, sizeof(int32_t) * TS_STATS_INTS,
                         hipMemcpyHostToDevice));
    } else {
        launch_reloc_rig(c, frame, h->d_map_xyz, h->d_map_desc, (int)h->map_n, h->d_rl_match, h->d_rl_corr, h->d_rl_stats,
                         h->d_rl_pose, h->d_rl_ransac, h->d_rl_hyp, h->d_rl_rig_pose, h->d_rl_rig_stats, s);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    double pose[TS_POSE_DOUBLES];
    int32_t st[TS_STATS_INTS];
    HIPCHK(hipMemcpy(pose, h->d_rl_rig_pose, sizeof(pose), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(st, h->d_rl_rig_stats, sizeof(st), hipMemcpyDeviceToHost));
    if (h->map_n == 0 || st[0] != 0)
        for (int i = 0; i < 16; ++i) pose[i] = (i % 5) == 0 ? 1.0 : 0.0;
    pose[12] = pose[13] = pose[14] = 0.0;   // k_rig_pose writes the 3x4 part
    pose[15] = 1.0;
    if (body_T_world) memcpy(body_T_world, pose, 16 * sizeof(double));
    if (cov) memcpy(cov, pose + 32, 36 * sizeof(double));
    if (stats) memcpy(stats, st, sizeof(st));
    if (pair_stats) HIPCHK(hipMemcpy(pair_stats, h->d_rl_stats, sizeof(int32_t) * TS_STATS_INTS * P, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

// -- loop closure: keyframe database, place recognition, verification, pose graph ---------------
int tslam_loop_init(tslam_handle* h, int max_keyframes, int signature) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (max_keyframes < 1 || max_keyframes > (1 << 16)) return fail(TSLAM_EINVAL, "max_keyframes must be in [1, 65536]");
    if (signature < 1 || signature > 256) return fail(TSLAM_EINVAL, "signature must be in [1, 256]");
    loop_worker_drain(h);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t K = h->g.K, cap = max_keyframes;
    int rc = dev_realloc(h, (void**)&h->d_lp_xyz, sizeof(double) * 3 * K * cap);
    if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_lp_desc, sizeof(uint32_t) * 8 * K * cap);
    if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_lp_n, sizeof(int32_t) * cap);
    if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_lp_votes, sizeof(int32_t) * cap);
    if (rc == TSLAM_OK) rc = ensure_reloc_scratch(h);
    if (rc != TSLAM_OK) return rc;
    for (void** p : {(void**)&h->d_lp_snap_kps, (void**)&h->d_lp_snap_kcount, (void**)&h->d_lp_snap_desc})
        if (*p) {   // snapshots follow the capacity: tslam_loop_auto allocates them again
            (void)hipFree(*p);
            h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), *p), h->allocs.end());
            *p = nullptr;
        }
    h->lp_auto = 0;
    h->lp_cap = max_keyframes;
    h->lp_S = signature;
    h->lp_count = 0;
    for (auto& j : h->lp_jobs) j.kind = 0;
    h->lp_store_armed = false;
    return TSLAM_OK;
}

static int loop_count(tslam_handle* h, int slot, int32_t* n) {
    HIPCHK(hipMemcpy(n, h->d_lp_n + slot, sizeof(int32_t), hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_loop_add_keyframe(tslam_handle* h, int pair, int64_t frame, int* slot, int* n_landmarks) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    if (h->lp_auto) return fail(TSLAM_ESTATE, "the submit path stores the keyframes (tslam_loop_auto)");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_loop_add_keyframe inside a batch");
    if (frame < 0 || frame >= h->frames_done || frame < h->frames_done - h->R)
        return fail(TSLAM_EINVAL, "frame is not resident in the ring");
    HIPCHK(hipSetDevice(h->device));
    if (loop_quiesce(h) != TSLAM_OK) return TSLAM_EHIP;
    const int sl = (int)(h->lp_count % h->lp_cap);
    const size_t K = h->g.K;
    const BatchCtx c = make_ctx(h);
    hipStream_t s = h->last_stream;
    launch_loop_store(c, pair, frame, h->d_lp_xyz + (size_t)sl * K * 3, h->d_lp_desc + (size_t)sl * K * 8, h->d_lp_n + sl, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    int32_t n = 0;
    if (loop_count(h, sl, &n) != TSLAM_OK) return TSLAM_EHIP;
    ++h->lp_count;
    if (slot) *slot = sl;
    if (n_landmarks) *n_landmarks = n;
    return TSLAM_OK;
}

int tslam_loop_read_keyframe(tslam_handle* h, int slot, double* xyz, uint32_t* desc, int* n) {
    if (!h || !h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    BA_FLUSH(h);
    if (slot < 0 || slot >= h->lp_cap) return fail(TSLAM_EINVAL, "slot out of range");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());   // the stores of every stream (tslam_loop_auto: the back stream)
    int32_t m = 0;
    if (loop_count(h, slot, &m) != TSLAM_OK) return TSLAM_EHIP;
    const size_t K = h->g.K;
    if (xyz && m) HIPCHK(hipMemcpy(xyz, h->d_lp_xyz + (size_t)slot * K * 3, sizeof(double) * 3 * m, hipMemcpyDeviceToHost));
    if (desc && m) HIPCHK(hipMemcpy(desc, h->d_lp_desc + (size_t)slot * K * 8, sizeof(uint32_t) * 8 * m, hipMemcpyDeviceToHost));
    if (n) *n = (int)m;
    return TSLAM_OK;
}

int tslam_loop_query(tslam_handle* h, int slot, int n_candidates, int32_t* votes) {
    if (!h || !h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    BA_FLUSH(h);
    if (slot < 0 || slot >= h->lp_cap) return fail(TSLAM_EINVAL, "slot out of range");
    if (n_candidates < 0 || n_candidates > h->lp_cap) return fail(TSLAM_EINVAL, "n_candidates out of range");
    if (n_candidates == 0) return TSLAM_OK;
    HIPCHK(hipSetDevice(h->device));
    if (loop_quiesce(h) != TSLAM_OK) return TSLAM_EHIP;
    hipStream_t s = h->last_stream;
    launch_loop_vote(h->d_lp_desc, h->d_lp_n, h->g.K, h->lp_S, slot, 0, std::numeric_limits<int>::max(), 1, n_candidates,
                     h->prm.max_hamming, h->prm.ratio_pct, h->d_lp_votes, s);
    HIPCHK(hipGetLastError());
    if (votes) HIPCHK(hipMemcpyAsync(votes, h->d_lp_votes, sizeof(int32_t) * n_candidates, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return TSLAM_OK;
}

int tslam_loop_verify(tslam_handle* h, int pair, int64_t frame, int slot, double* T_qc, double* cov, int32_t* stats) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    if (slot < 0 || slot >= h->lp_cap) return fail(TSLAM_EINVAL, "slot out of range");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_loop_verify inside a batch");
    if (frame < 0 || frame >= h->frames_done || frame < h->frames_done - h->R)
        return fail(TSLAM_EINVAL, "frame is not resident in the ring");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    int32_t m = 0;
    if (loop_count(h, slot, &m) != TSLAM_OK) return TSLAM_EHIP;
    const size_t K = h->g.K;
    return reloc_solve(h, pair, frame, h->d_lp_xyz + (size_t)slot * K * 3, h->d_lp_desc + (size_t)slot * K * 8, m, T_qc,
                       cov, stats);
}

// -- asynchronous loop closure (tslam_loop_auto / tslam_loop_job_*) ------------------------------
static int pose_graph_reserve(tslam_handle* h, int n_nodes, int n_edges);

int tslam_loop_auto(tslam_handle* h, int interval) {
    if (!h || interval < 0) return fail(TSLAM_EINVAL, "bad handle or interval");
    BA_FLUSH(h);
    if (!h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_loop_auto inside a batch");
    if (h->sh_world > 1 || h->sh_comm) return fail(TSLAM_ESTATE, "tslam_loop_auto takes an unsharded handle");
    if (h->lp_cap % h->P) return fail(TSLAM_EINVAL, "max_keyframes of tslam_loop_init must be a multiple of the pairs");
    HIPCHK(hipSetDevice(h->device));
    if (interval && !h->d_lp_snap_kps) {
        const size_t K = h->g.K, cap = h->lp_cap;
        int rc = dev_alloc(h, (void**)&h->d_lp_snap_kps, sizeof(uint32_t) * 2 * K * cap);
        if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_lp_snap_kcount, sizeof(int32_t) * TS_MAX_LEVELS * cap);
        if (rc == TSLAM_OK) rc = dev_alloc(h, (void**)&h->d_lp_snap_desc, sizeof(uint32_t) * 8 * K * cap);
        if (rc != TSLAM_OK) return rc;
    }
    if (interval && !h->d_lp_pos) {
        const int rc = dev_alloc(h, (void**)&h->d_lp_pos, sizeof(int64_t));
        if (rc != TSLAM_OK) return rc;
    }
    if (interval && h->d_lp_pos) HIPCHK(hipMemset(h->d_lp_pos, 0, sizeof(int64_t)));   // (dev_alloc synchronised)
    if (interval) {   // a span solve covers at most the ring's cap_k nodes (and one loop edge per node)
        const int nn = std::min(1024, h->lp_cap / h->P);
        const int rc = pose_graph_reserve(h, std::max(nn, 2), 2 * std::max(nn, 2));
        if (rc != TSLAM_OK) return rc;
    }
    HIPCHK(hipDeviceSynchronize());
    if (interval && !h->lp_ev_store) HIPCHK(hipEventCreateWithFlags(&h->lp_ev_store, hipEventDisableTiming));
    h->lp_auto = interval;
    return TSLAM_OK;
}

// Grows geometrically (and to at least 4 KiB): a job slot's buffer is reallocated O(log) times as
// the vote window or the pose-graph span grows, not on every job (a pinned allocation and free
// cost ~0.2 ms of the submitting thread).
static int pinned_reserve(tslam_handle* h, void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return TSLAM_OK;
    bytes = std::max({bytes, 2 * *cap, (size_t)4096});
    if (*p) {
        (void)hipHostFree(*p);
        h->host_allocs.erase(std::remove(h->host_allocs.begin(), h->host_allocs.end(), *p), h->host_allocs.end());
        *p = nullptr;
        *cap = 0;
    }
    HIPCHK(hipHostMalloc(p, bytes, hipHostMallocDefault));
    h->host_allocs.push_back(*p);
    *cap = bytes;
    return TSLAM_OK;
}

// A job slot (the loop stream created on first use).  The caller stages the inputs; the worker
// makes the loop stream wait for the newest batch's keyframe stores (so a job sees every entry of
// every batch submitted before it), runs `work` and records the job's event.
static int job_begin(tslam_handle* h, int kind, tslam_handle::LoopJob** out) {
    if (!h->lp_stream) HIPCHK(hipStreamCreateWithFlags(&h->lp_stream, hipStreamNonBlocking));
    auto& j = h->lp_jobs[h->lp_job_next % 64];
    if (j.kind) return fail(TSLAM_ESTATE, "64 loop jobs are unreturned (tslam_loop_job_poll)");
    if (!j.ev) HIPCHK(hipEventCreateWithFlags(&j.ev, hipEventDisableTiming));
    j.kind = kind;
    j.id = h->lp_job_next;
    j.posted = 0;
    j.err.clear();
    *out = &j;
    return TSLAM_OK;
}

static int job_post(tslam_handle* h, tslam_handle::LoopJob& j, std::function<hipError_t()> work, int64_t* id) {
    const bool wait_store = h->lp_store_armed;
    tslam_handle::LoopJob* jp = &j;
    loop_worker_post(h, [h, jp, wait_store, work = std::move(work)] {
        hipError_t e = wait_store ? hipStreamWaitEvent(h->lp_stream, h->lp_ev_store, 0) : hipSuccess;
        if (e == hipSuccess) e = work();
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(jp->ev, h->lp_stream);
        std::lock_guard<std::mutex> lk(h->lp_worker->mu);
        jp->posted = e == hipSuccess ? 1 : -1;
        if (e != hipSuccess) jp->err = std::string("loop job: ") + hipGetErrorString(e);
    });
    ++h->lp_job_next;
    if (id) *id = j.id;
    return TSLAM_OK;
}

int tslam_loop_job_vote(tslam_handle* h, int query, int64_t k0, int n_kf, int64_t* job) {
    if (!h || !h->lp_cap) return fail(TSLAM_ESTATE, "loop database not initialised (tslam_loop_init)");
    BA_FLUSH(h);
    if (h->lp_cap % h->P) return fail(TSLAM_ESTATE, "the database is not keyframe-major over the pairs");
    const int capk = h->lp_cap / h->P;
    if (query < 0 || query >= h->lp_cap || k0 < 0 || n_kf < 0 || n_kf > capk)
        return fail(TSLAM_EINVAL, "query entry or keyframe range out of range");
    HIPCHK(hipSetDevice(h->device));
    tslam_handle::LoopJob* j = nullptr;
    int rc = job_begin(h, 1, &j);
    if (rc != TSLAM_OK) return rc;
    const int n = n_kf * h->P;
    j->n_out = n;
    // sized for the whole database at once: the vote window grows with every keyframe
    if ((rc = pinned_reserve(h, &j->out, &j->out_cap, sizeof(int32_t) * std::max(n, h->lp_cap))) != TSLAM_OK) {
        j->kind = 0;
        return rc;
    }
    const int K = h->g.K, S = h->lp_S, P = h->P, mh = h->prm.max_hamming, rp = h->prm.ratio_pct;
    const uint32_t* desc = h->d_lp_desc;
    const int32_t* cnt = h->d_lp_n;
    int32_t* votes = h->d_lp_votes;
    void* out = j->out;
    return job_post(h, *j, [=]() -> hipError_t {
        if (!n) return hipSuccess;
        launch_loop_vote(desc, cnt, K, S, query, k0, capk, P, n, mh, rp, votes, h->lp_stream);
        return hipMemcpyAsync(out, votes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->lp_stream);
    }, job);
}

int tslam_loop_job_verify(tslam_handle* h, int pair, int64_t frame, int query, int cand, int64_t* job) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->lp_cap || !h->d_lp_snap_kps) return fail(TSLAM_ESTATE, "no keyframe snapshots (tslam_loop_auto)");
    if (query < 0 || query >= h->lp_cap || cand < 0 || cand >= h->lp_cap || frame < 0)
        return fail(TSLAM_EINVAL, "entry or frame out of range");
    // entry (position mod cap_k) * P + p holds pair p's view: its snapshot must be solved with
    // that pair's calibration
    if (query % h->P != pair) return fail(TSLAM_EINVAL, "query entry is not a view of `pair` (entry % n_pairs)");
    HIPCHK(hipSetDevice(h->device));
    tslam_handle::LoopJob* j = nullptr;
    int rc = job_begin(h, 2, &j);
    if (rc != TSLAM_OK) return rc;
    const size_t pose_b = sizeof(double) * TS_POSE_DOUBLES, stat_b = sizeof(int32_t) * TS_STATS_INTS;
    if ((rc = pinned_reserve(h, &j->out, &j->out_cap, pose_b + stat_b)) != TSLAM_OK) {
        j->kind = 0;
        return rc;
    }
    const size_t K = h->g.K;
    const RelocQuery q{h->d_lp_snap_kps + (size_t)query * K * 2, h->d_lp_snap_kcount + (size_t)query * TS_MAX_LEVELS,
                       h->d_lp_snap_desc + (size_t)query * K * 8};
    const BatchCtx c = make_ctx(h);   // built here: the worker must not read the handle's batch state
    const double* xyz = h->d_lp_xyz + (size_t)cand * K * 3;
    const uint32_t* desc = h->d_lp_desc + (size_t)cand * K * 8;
    const int32_t* dM = h->d_lp_n + cand;
    void* out = j->out;
    return job_post(h, *j, [=]() -> hipError_t {
        launch_reloc_query(c, pair, frame, q, xyz, desc, 0, dM, h->d_rl_match, h->d_rl_corr, h->d_rl_stats, h->d_rl_pose,
                           h->d_rl_ransac, h->d_rl_hyp, h->lp_stream);
        hipError_t e = hipMemcpyAsync(out, h->d_rl_pose, pose_b, hipMemcpyDeviceToHost, h->lp_stream);
        if (e == hipSuccess) e = hipMemcpyAsync((char*)out + pose_b, h->d_rl_stats, stat_b, hipMemcpyDeviceToHost, h->lp_stream);
        return e;
    }, job);
}

// -- RGB-D dense mapping: TSDF integration -------------------------------------------------------
int tslam_tsdf_init(tslam_handle* h, const double* origin, const int32_t* dims, double voxel_size, double trunc_vox,
                    double max_dist, double max_weight) {
    if (!h || !origin || !dims) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (dims[0] < 1 || dims[1] < 1 || dims[2] < 1 || (int64_t)dims[0] * dims[1] * dims[2] > ((int64_t)1 << 31))
        return fail(TSLAM_EINVAL, "dims must be >= 1 with at most 2^31 voxels");
    if (!(voxel_size > 0.0) || !(trunc_vox > 0.0) || !(max_dist > 0.0) || !(max_weight >= 1.0))
        return fail(TSLAM_EINVAL, "voxel_size, trunc_vox, max_dist must be > 0 and max_weight >= 1");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)dims[0] * dims[1] * dims[2];
    TsdfArgs& a = h->tsdf;
    int rc = dev_realloc(h, (void**)&a.tsdf, sizeof(float) * nv);
    if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&a.weight, sizeof(float) * nv);
    if (rc == TSLAM_OK && h->tsdf_color) {
        rc = dev_realloc(h, (void**)&a.col, sizeof(float) * 3 * nv);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&a.col_w, sizeof(float) * nv);
    }
    if (rc == TSLAM_OK && !h->d_tsdf_poses) rc = dev_alloc(h, (void**)&h->d_tsdf_poses, sizeof(double) * TSDF_MAX_FRAMES * TSDF_POSE);
    if (rc == TSLAM_OK && !h->d_tsdf_wTc) rc = dev_alloc(h, (void**)&h->d_tsdf_wTc, sizeof(double) * TSDF_MAX_FRAMES * 16);
    if (rc != TSLAM_OK) return rc;
    a.nx = dims[0];
    a.ny = dims[1];
    a.nz = dims[2];
    a.ox = origin[0];
    a.oy = origin[1];
    a.oz = origin[2];
    a.s = voxel_size;
    a.trunc = trunc_vox * voxel_size;
    a.max_dist = max_dist;
    a.max_weight = max_weight;
    h->tsdf_on = true;
    h->esdf_valid = false;   // outputs of the previous volume are gone
    h->mesh_n = 0;
    return TSLAM_OK;
}

static int tsdf_integrate(tslam_handle* h, int pair, const void* color, const void* depth, int64_t stride_bytes,
                          int n_frames, int64_t first_frame, const double* world_T_cam, void* stream);

int tslam_tsdf_integrate(tslam_handle* h, int pair, const void* depth, int64_t stride_bytes, int n_frames,
                         int64_t first_frame, const double* world_T_cam, void* stream) {
    return tsdf_integrate(h, pair, nullptr, depth, stride_bytes, n_frames, first_frame, world_T_cam, stream);
}

int tslam_tsdf_integrate_rgbd(tslam_handle* h, int pair, const void* color, const void* depth, int64_t stride_bytes,
                              int n_frames, int64_t first_frame, const double* world_T_cam, void* stream) {
    if (!color) return fail(TSLAM_EINVAL, "null colour images");
    if (h && !h->tsdf_color) return fail(TSLAM_ESTATE, "no colour layer (tslam_tsdf_color before tslam_tsdf_init)");
    return tsdf_integrate(h, pair, color, depth, stride_bytes, n_frames, first_frame, world_T_cam, stream);
}

int tslam_tsdf_color(tslam_handle* h, int enable) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    if (h->tsdf_on && (enable != 0) != h->tsdf_color) return fail(TSLAM_ESTATE, "tslam_tsdf_color before tslam_tsdf_init");
    h->tsdf_color = enable != 0;
    return TSLAM_OK;
}

static int tsdf_integrate(tslam_handle* h, int pair, const void* color, const void* depth, int64_t stride_bytes,
                          int n_frames, int64_t first_frame, const double* world_T_cam, void* stream) {
    if (!h || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    if (!depth || n_frames < 0 || (n_frames > 1 && stride_bytes < 2LL * h->W * h->H)) return fail(TSLAM_EINVAL, "bad depth / stride");
    if (h->in_batch) return fail(TSLAM_ESTATE, "tslam_tsdf_integrate inside a batch");
    int f0 = 0;
    if (!world_T_cam) {   // device poses: frames of the last batch
        f0 = (int)(first_frame - h->cur_g0);
        if (first_frame < h->cur_g0 || f0 + n_frames > h->cur_n)
            return fail(TSLAM_EINVAL, "device poses: frames must belong to the last batch");
    }
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->last_stream;
    const BatchCtx c = make_ctx(h);
    const int cam = c.cpp * pair;
    TsdfArgs a = h->tsdf;
    a.W = h->W;
    a.H = h->H;
    a.fx = h->calib[pair].fx;
    a.fy = h->calib[pair].fy;
    a.cx = h->calib[pair].cx;
    a.cy = h->calib[pair].cy;
    a.map = ((h->map_mask >> cam) & 1u) ? h->d_maps + (size_t)cam * h->W * h->H * 2 : nullptr;
    a.stride = stride_bytes;
    if (!color) a.col = a.col_w = nullptr;   // the colour layer keeps its state without colour input
    for (int b0 = 0; b0 < n_frames; b0 += TSDF_MAX_FRAMES) {
        a.n = std::min(TSDF_MAX_FRAMES, n_frames - b0);
        a.depth = static_cast<const uint8_t*>(depth) + (size_t)b0 * stride_bytes;
        a.color = color ? static_cast<const uint8_t*>(color) + (size_t)b0 * stride_bytes : nullptr;
        const double* wtc = nullptr;
        if (world_T_cam) {
            HIPCHK(hipMemcpyAsync(h->d_tsdf_wTc, world_T_cam + (size_t)16 * b0, sizeof(double) * 16 * a.n,
                                  hipMemcpyHostToDevice, s));
            wtc = h->d_tsdf_wTc;
        }
        launch_tsdf(c, pair, f0 + b0, wtc, a, h->d_tsdf_poses, s);
        HIPCHK(hipGetLastError());
        if (world_T_cam) HIPCHK(hipStreamSynchronize(s));   // the staged host poses are reused
    }
    return TSLAM_OK;
}

int tslam_tsdf_read(tslam_handle* h, float* tsdf, float* weight) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    BA_FLUSH(h);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
    if (tsdf) HIPCHK(hipMemcpy(tsdf, h->tsdf.tsdf, sizeof(float) * nv, hipMemcpyDeviceToHost));
    if (weight) HIPCHK(hipMemcpy(weight, h->tsdf.weight, sizeof(float) * nv, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_tsdf_read_color(tslam_handle* h, float* rgb, float* weight) {
    if (!h || !h->tsdf_on || !h->tsdf_color) return fail(TSLAM_ESTATE, "no colour layer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
    if (rgb) HIPCHK(hipMemcpy(rgb, h->tsdf.col, sizeof(float) * 3 * nv, hipMemcpyDeviceToHost));
    if (weight) HIPCHK(hipMemcpy(weight, h->tsdf.col_w, sizeof(float) * nv, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_tsdf_write_color(tslam_handle* h, const float* rgb, const float* weight) {
    if (!h || !h->tsdf_on || !h->tsdf_color) return fail(TSLAM_ESTATE, "no colour layer");
    if (!rgb || !weight) return fail(TSLAM_EINVAL, "null colour volume");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
    HIPCHK(hipMemcpy(h->tsdf.col, rgb, sizeof(float) * 3 * nv, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->tsdf.col_w, weight, sizeof(float) * nv, hipMemcpyHostToDevice));
    return TSLAM_OK;
}

int tslam_tsdf_write(tslam_handle* h, const float* tsdf, const float* weight) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    BA_FLUSH(h);
    if (!tsdf || !weight) return fail(TSLAM_EINVAL, "null volume");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
    HIPCHK(hipMemcpy(h->tsdf.tsdf, tsdf, sizeof(float) * nv, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->tsdf.weight, weight, sizeof(float) * nv, hipMemcpyHostToDevice));
    h->esdf_valid = false;
    return TSLAM_OK;
}

// -- dense-map outputs: marching-cubes mesh, ESDF, 2-D ESDF slice (k_dense.hip) ------------------
static DenseArgs dense_args(const tslam_handle* h, double min_weight) {
    const TsdfArgs& t = h->tsdf;
    DenseArgs a{};
    a.tsdf = t.tsdf;
    a.weight = t.weight;
    a.nx = t.nx;
    a.ny = t.ny;
    a.nz = t.nz;
    a.n_cubes = (t.nx > 1 && t.ny > 1 && t.nz > 1) ? (uint32_t)((int64_t)(t.nx - 1) * (t.ny - 1) * (t.nz - 1)) : 0u;
    a.n_voxels = (int64_t)t.nx * t.ny * t.nz;
    a.ox = t.ox;
    a.oy = t.oy;
    a.oz = t.oz;
    a.s = t.s;
    a.sf = (float)t.s;
    a.min_weight = (float)min_weight;
    a.color = h->tsdf_color ? t.col : nullptr;
    return a;
}

static int grow(tslam_handle* h, void** p, size_t* cap, size_t need) {
    if (*cap >= need && *p) return TSLAM_OK;
    const int rc = dev_realloc(h, p, need);
    *cap = rc == TSLAM_OK ? need : 0;
    return rc;
}

int tslam_mesh_extract(tslam_handle* h, double min_weight, int64_t* n_tris, void* stream) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    BA_FLUSH(h);
    if (!(min_weight >= 0.0)) return fail(TSLAM_EINVAL, "min_weight must be >= 0");
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->last_stream;
    const DenseArgs a = dense_args(h, min_weight);
    h->mesh_n = 0;
    if (a.n_cubes == 0) {
        if (n_tris) *n_tris = 0;
        return TSLAM_OK;
    }
    const size_t nb = (a.n_cubes + 255) / 256;
    size_t cap = h->mesh_cubes_cap;
    if (cap < a.n_cubes) {   // the three scratch arrays follow the cube count
        size_t c0 = 0, c1 = 0, c2 = 0;
        int rc = grow(h, (void**)&h->d_mesh_cfg, &c0, a.n_cubes);
        if (rc == TSLAM_OK) rc = grow(h, (void**)&h->d_mesh_bsum, &c1, sizeof(uint32_t) * nb);
        if (rc == TSLAM_OK) rc = grow(h, (void**)&h->d_mesh_boff, &c2, sizeof(uint64_t) * (nb + 1));
        if (rc != TSLAM_OK) return rc;
        h->mesh_cubes_cap = a.n_cubes;
    }
    launch_mesh_count(a, h->d_mesh_cfg, h->d_mesh_bsum, h->d_mesh_boff, h->d_mesh_boff + nb, s);
    HIPCHK(hipGetLastError());
    uint64_t total = 0;   // the buffer is sized to the count: one small read back
    HIPCHK(hipMemcpyAsync(&total, h->d_mesh_boff + nb, sizeof(total), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if ((int64_t)total > h->mesh_tris_cap || (a.color && !h->d_mesh_cols)) {
        size_t c = 0, c2 = 0;
        const int64_t want = std::max((int64_t)total + (int64_t)total / 4 + 1024, h->mesh_tris_cap);
        int rc = grow(h, (void**)&h->d_mesh_tris, &c, sizeof(float) * 9 * (size_t)want);
        if (rc == TSLAM_OK && a.color) rc = grow(h, (void**)&h->d_mesh_cols, &c2, sizeof(float) * 9 * (size_t)want);
        if (rc != TSLAM_OK) return rc;
        h->mesh_tris_cap = want;
    }
    launch_mesh_emit(a, h->d_mesh_cfg, h->d_mesh_boff, h->d_mesh_tris, h->d_mesh_cols, h->mesh_tris_cap, s);
    HIPCHK(hipGetLastError());
    h->mesh_n = (int64_t)total;
    if (n_tris) *n_tris = (int64_t)total;
    return TSLAM_OK;
}

int tslam_mesh_read_colors(tslam_handle* h, float* colors, int64_t max_tris) {
    if (!h || !h->tsdf_on || !h->tsdf_color || !h->d_mesh_cols) return fail(TSLAM_ESTATE, "no colour layer mesh");
    if (max_tris < 0 || (max_tris > 0 && !colors)) return fail(TSLAM_EINVAL, "bad buffer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const int64_t n = std::min(max_tris, h->mesh_n);
    if (n > 0) HIPCHK(hipMemcpy(colors, h->d_mesh_cols, sizeof(float) * 9 * (size_t)n, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_mesh_read(tslam_handle* h, float* tris, int64_t max_tris) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    if (max_tris < 0 || (max_tris > 0 && !tris)) return fail(TSLAM_EINVAL, "bad buffer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const int64_t n = std::min(max_tris, h->mesh_n);
    if (n > 0) HIPCHK(hipMemcpy(tris, h->d_mesh_tris, sizeof(float) * 9 * (size_t)n, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

// f32 distance of every squared voxel distance 0..R^2 (sqrt in f32, times s in f32, IEEE on the host)
static int dist_table(tslam_handle* h, int R, double s) {
    if (h->dist_tab_R == R && h->dist_tab_s == s && h->d_dist_tab) return TSLAM_OK;
    const size_t n = (size_t)R * R + 1;
    std::vector<float> tab(n);
    const float sf = (float)s;
    for (size_t d = 0; d < n; ++d) tab[d] = std::sqrt((float)d) * sf;
    const int rc = dev_realloc(h, (void**)&h->d_dist_tab, sizeof(float) * n);
    if (rc != TSLAM_OK) return rc;
    HIPCHK(hipMemcpy(h->d_dist_tab, tab.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    h->dist_tab_R = R;
    h->dist_tab_s = s;
    return TSLAM_OK;
}

static int esdf_setup(tslam_handle* h, double max_dist, double site_vox, double min_weight, size_t cells, DenseArgs* a,
                      int* R) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    if (!(max_dist > 0.0) || !(site_vox >= 0.0) || !(min_weight >= 0.0))
        return fail(TSLAM_EINVAL, "max_dist must be > 0, site_vox and min_weight >= 0");
    const double r = std::floor(max_dist / h->tsdf.s + 1e-9);
    if (r < 0.0 || r > 2048.0) return fail(TSLAM_EINVAL, "max_dist / voxel_size must be at most 2048 voxels");
    HIPCHK(hipSetDevice(h->device));
    *R = (int)r;
    *a = dense_args(h, min_weight);
    a->site_dist = (float)(site_vox * h->tsdf.s);
    a->max_dist = (float)max_dist;
    a->cap = *R * *R + 1;
    int rc = dist_table(h, *R, h->tsdf.s);
    if (rc == TSLAM_OK && h->edt_cap < cells) {
        size_t c0 = 0, c1 = 0;
        rc = grow(h, (void**)&h->d_edt[0], &c0, sizeof(int32_t) * cells);
        if (rc == TSLAM_OK) rc = grow(h, (void**)&h->d_edt[1], &c1, sizeof(int32_t) * cells);
        h->edt_cap = rc == TSLAM_OK ? cells : 0;
    }
    return rc;
}

int tslam_esdf_compute(tslam_handle* h, double max_dist, double site_vox, double min_weight, void* stream) {
    DenseArgs a;
    int R = 0;
    const size_t nv = h && h->tsdf_on ? (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz : 0;
    int rc = esdf_setup(h, max_dist, site_vox, min_weight, nv, &a, &R);
    if (rc == TSLAM_OK) rc = grow(h, (void**)&h->d_esdf, &h->esdf_cap, sizeof(float) * nv);
    if (rc != TSLAM_OK) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->last_stream;
    launch_esdf(a, R, h->d_dist_tab, h->d_edt[0], h->d_edt[1], h->d_esdf, s);
    HIPCHK(hipGetLastError());
    h->esdf_valid = true;
    return TSLAM_OK;
}

int tslam_esdf_read(tslam_handle* h, float* esdf) {
    if (!h || !h->tsdf_on || !h->esdf_valid) return fail(TSLAM_ESTATE, "no ESDF (tslam_esdf_compute)");
    if (!esdf) return fail(TSLAM_EINVAL, "null buffer");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const size_t nv = (size_t)h->tsdf.nx * h->tsdf.ny * h->tsdf.nz;
    HIPCHK(hipMemcpy(esdf, h->d_esdf, sizeof(float) * nv, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_esdf_slice(tslam_handle* h, int y0, int y1, double max_dist, double site_vox, double min_weight, float* out) {
    if (!h || !h->tsdf_on) return fail(TSLAM_ESTATE, "no TSDF volume (tslam_tsdf_init)");
    if (!out || y0 < 0 || y1 <= y0 || y1 > h->tsdf.ny) return fail(TSLAM_EINVAL, "need 0 <= y0 < y1 <= ny and a buffer");
    DenseArgs a;
    int R = 0;
    const size_t nc = (size_t)h->tsdf.nx * h->tsdf.nz;
    int rc = esdf_setup(h, max_dist, site_vox, min_weight, nc, &a, &R);
    if (rc == TSLAM_OK && h->slice_cap < nc) {
        size_t c0 = 0, c1 = 0;
        rc = grow(h, (void**)&h->d_slice_obs, &c0, nc);
        if (rc == TSLAM_OK) rc = grow(h, (void**)&h->d_slice, &c1, sizeof(float) * nc);
        h->slice_cap = rc == TSLAM_OK ? nc : 0;
    }
    if (rc != TSLAM_OK) return rc;
    hipStream_t s = h->last_stream;
    launch_esdf_slice(a, y0, y1, R, h->d_dist_tab, h->d_edt[0], h->d_edt[1], h->d_slice_obs, h->d_slice, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(out, h->d_slice, sizeof(float) * nc, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

// Pose-graph scratch for n_nodes / n_edges.  Growth reallocates (and synchronises the device), so
// tslam_loop_auto reserves the largest span solve up front.
static int pose_graph_reserve(tslam_handle* h, int n_nodes, int n_edges) {
    const int np = (6 * (n_nodes - 1) + 31) / 32 * 32;
    int rc = TSLAM_OK;
    if (n_nodes > h->pg_nodes || n_edges > h->pg_edges || np > h->pg_np) {
        // growth frees the d_pg_* buffers that queued pose-graph jobs read when the worker issues
        // them (and their kernels on the loop stream): drain the worker and the stream first, so
        // no job holds an old pointer and no other thread reads the fields being replaced
        loop_worker_drain(h);
        if (h->lp_stream) HIPCHK(hipStreamSynchronize(h->lp_stream));
    }
    if (!h->d_pg_cost && (rc = dev_alloc(h, (void**)&h->d_pg_cost, sizeof(double))) != TSLAM_OK) return rc;
    if (n_nodes > h->pg_nodes) {
        rc = dev_realloc(h, (void**)&h->d_pg_T, sizeof(double) * 16 * n_nodes);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_adj_off, sizeof(int32_t) * (n_nodes + 1));
        if (rc != TSLAM_OK) return rc;
        h->pg_nodes = n_nodes;
    }
    if (n_edges > h->pg_edges) {
        rc = dev_realloc(h, (void**)&h->d_pg_Z, sizeof(double) * 16 * n_edges);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_info, sizeof(double) * 36 * n_edges);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_terms, sizeof(double) * 128 * n_edges);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_edges, sizeof(int32_t) * 2 * n_edges);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_adj, sizeof(int32_t) * 2 * n_edges);
        if (rc != TSLAM_OK) return rc;
        h->pg_edges = n_edges;
    }
    if (np > h->pg_np) {
        rc = dev_realloc(h, (void**)&h->d_pg_H, sizeof(double) * (size_t)np * np);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_ftile, sizeof(int32_t) * (np / 32));
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_g, sizeof(double) * np);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_delta, sizeof(double) * np);
        if (rc == TSLAM_OK) rc = dev_realloc(h, (void**)&h->d_pg_Ld, sizeof(double) * np);
        if (rc != TSLAM_OK) return rc;
        h->pg_np = np;
    }
    return TSLAM_OK;
}

// The pose-graph solve as a loop job: validation, the CSR incidence and the matrix profile on the
// host, every input copied into the job's pinned staging at the call, the iterations on the loop
// stream, the poses and the per-edge cost terms back into pinned memory.
int tslam_loop_job_pose_graph(tslam_handle* h, int n_nodes, const double* world_T_node, int n_edges, const int32_t* edges,
                              const double* meas, const double* info, int iters, int64_t* job) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (n_nodes < 1 || n_nodes > 1024) return fail(TSLAM_EINVAL, "n_nodes must be in [1, 1024]");
    if (n_edges < 0 || (n_edges && (!edges || !meas || !info)) || !world_T_node || iters < 0)
        return fail(TSLAM_EINVAL, "bad argument");
    // incident-edge lists (CSR, by edge index) of every node; every free node needs an edge
    std::vector<int32_t> off(n_nodes + 1, 0), adj(2 * (size_t)n_edges);
    for (int k = 0; k < n_edges; ++k) {
        const int a = edges[2 * k], b = edges[2 * k + 1];
        if (a < 0 || a >= n_nodes || b < 0 || b >= n_nodes || a == b) return fail(TSLAM_EINVAL, "bad edge");
        ++off[a + 1];
        ++off[b + 1];
    }
    for (int i = 0; i < n_nodes; ++i) off[i + 1] += off[i];
    {
        std::vector<int32_t> fill(off.begin(), off.end() - 1);
        for (int k = 0; k < n_edges; ++k) {
            adj[fill[edges[2 * k]]++] = (k << 1);
            adj[fill[edges[2 * k + 1]]++] = (k << 1) | 1;
        }
    }
    for (int i = 1; i < n_nodes; ++i)
        if (off[i + 1] == off[i]) return fail(TSLAM_EINVAL, "a free node has no edge");
    HIPCHK(hipSetDevice(h->device));
    const int n = 6 * (n_nodes - 1), np = (n + 31) / 32 * 32, nt = np / 32;
    // profile of the normal matrix: row block of node p (>= 1) starts at its lowest free
    // neighbour (or itself); ftile[I] = first nonzero tile column of tile row I
    std::vector<int32_t> ftile(std::max(nt, 1));
    for (int I = 0; I < nt; ++I) ftile[I] = I;
    for (int p = 1; p < n_nodes; ++p) {
        int lo = p;
        for (int i = off[p]; i < off[p + 1]; ++i) {
            const int k = adj[i] >> 1, other = edges[2 * k + ((adj[i] & 1) ? 0 : 1)];
            if (other >= 1) lo = std::min(lo, other);
        }
        const int col = 6 * (lo - 1) / 32;
        for (int r = 6 * (p - 1); r < 6 * p; ++r) ftile[r / 32] = std::min(ftile[r / 32], col);
    }
    int rc = pose_graph_reserve(h, n_nodes, n_edges);
    if (rc != TSLAM_OK) return rc;
    tslam_handle::LoopJob* j = nullptr;
    if ((rc = job_begin(h, 3, &j)) != TSLAM_OK) return rc;
    j->n_out = n_nodes;
    j->n_edges = n_edges;
    // staging: T | Z | info | off | ftile | edges | adj (doubles first, 8-byte aligned)
    const size_t bT = sizeof(double) * 16 * n_nodes, bZ = sizeof(double) * 16 * n_edges, bI = sizeof(double) * 36 * n_edges;
    const size_t bO = sizeof(int32_t) * (n_nodes + 1), bF = sizeof(int32_t) * nt, bE = sizeof(int32_t) * 2 * n_edges;
    const size_t out_b = bT + sizeof(double);
    if ((rc = pinned_reserve(h, &j->in, &j->in_cap, bT + bZ + bI + bO + bF + 2 * bE)) != TSLAM_OK ||
        (rc = pinned_reserve(h, &j->out, &j->out_cap, out_b)) != TSLAM_OK) {
        j->kind = 0;
        return rc;
    }
    char* st = (char*)j->in;
    memcpy(st, world_T_node, bT);
    if (n_edges) {
        memcpy(st + bT, meas, bZ);
        memcpy(st + bT + bZ, info, bI);
        memcpy(st + bT + bZ + bI + bO + bF, edges, bE);
        memcpy(st + bT + bZ + bI + bO + bF + bE, adj.data(), bE);
    }
    memcpy(st + bT + bZ + bI, off.data(), bO);
    if (nt) memcpy(st + bT + bZ + bI + bO, ftile.data(), bF);
    void* out = j->out;
    return job_post(h, *j, [=]() -> hipError_t {
        hipStream_t s = h->lp_stream;
        hipError_t e = hipMemcpyAsync(h->d_pg_T, st, bT, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(h->d_pg_adj_off, st + bT + bZ + bI, bO, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && nt) e = hipMemcpyAsync(h->d_pg_ftile, st + bT + bZ + bI + bO, bF, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && n_edges) {
            e = hipMemcpyAsync(h->d_pg_Z, st + bT, bZ, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipMemcpyAsync(h->d_pg_info, st + bT + bZ, bI, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipMemcpyAsync(h->d_pg_edges, st + bT + bZ + bI + bO + bF, bE, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipMemcpyAsync(h->d_pg_adj, st + bT + bZ + bI + bO + bF + bE, bE, hipMemcpyHostToDevice, s);
        }
        if (e != hipSuccess) return e;
        if (n > 0)
            for (int it = 0; it < iters; ++it)
                launch_pose_graph_iteration(h->d_pg_T, h->d_pg_edges, h->d_pg_Z, h->d_pg_info, n_nodes, n_edges,
                                            h->d_pg_adj_off, h->d_pg_adj, h->d_pg_ftile, h->d_pg_terms, h->d_pg_H, h->d_pg_g,
                                            h->d_pg_delta, h->d_pg_Ld, s);
        // the cost (sum of the edges' e^T info e in edge order) reduced on the device: 8 bytes back
        launch_pose_graph_cost(h->d_pg_T, h->d_pg_edges, h->d_pg_Z, h->d_pg_info, n_edges, h->d_pg_terms, h->d_pg_cost, s);
        e = hipMemcpyAsync((char*)out + bT, h->d_pg_cost, sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(out, h->d_pg_T, bT, hipMemcpyDeviceToHost, s);
        return e;
    }, job);
}

int tslam_loop_job_poll(tslam_handle* h, int64_t id, int block, int32_t* votes, double* T_qc, double* cov,
                        int32_t* stats, double* world_T_node, double* cost) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    auto& j = h->lp_jobs[(size_t)(id > 0 ? id : 0) % 64];
    if (id <= 0 || !j.kind || j.id != id) return fail(TSLAM_ESTATE, "unknown or already returned loop job");
    HIPCHK(hipSetDevice(h->device));
    {   // the worker may not have issued it yet
        std::unique_lock<std::mutex> lk(h->lp_worker->mu);
        if (j.posted == 0) {
            if (!block) return 0;
            h->lp_worker->cv.wait(lk, [&] { return j.posted != 0; });
        }
        if (j.posted < 0) {
            j.kind = 0;
            return fail(TSLAM_EHIP, j.err);
        }
    }
    if (block) {
        HIPCHK(hipEventSynchronize(j.ev));
    } else {
        const hipError_t q = hipEventQuery(j.ev);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return fail(TSLAM_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    const int kind = j.kind;
    j.kind = 0;   // returned: the slot is free whatever follows
    if (kind == 1) {
        if (votes && j.n_out) memcpy(votes, j.out, sizeof(int32_t) * j.n_out);
    } else if (kind == 2) {
        double pose[TS_POSE_DOUBLES];
        int32_t st[TS_STATS_INTS];
        memcpy(pose, j.out, sizeof(pose));
        memcpy(st, (const char*)j.out + sizeof(pose), sizeof(st));
        if (st[0] != 0)   // as reloc_solve: identity when the verification failed
            for (int i = 0; i < 16; ++i) pose[i] = (i % 5) == 0 ? 1.0 : 0.0;
        pose[12] = pose[13] = pose[14] = 0.0;   // k_refine writes the 3x4 part only
        pose[15] = 1.0;
        if (T_qc) memcpy(T_qc, pose, 16 * sizeof(double));
        if (cov) memcpy(cov, pose + 32, 36 * sizeof(double));
        if (stats) memcpy(stats, st, sizeof(st));
    } else {
        const double* T = (const double*)j.out;
        for (int i = 0; i < 16 * j.n_out; ++i)
            if (!std::isfinite(T[i])) return fail(TSLAM_ESINGULAR, "pose graph: normal matrix not positive definite");
        if (world_T_node) memcpy(world_T_node, T, sizeof(double) * 16 * j.n_out);
        if (cost) *cost = T[16 * (size_t)j.n_out];
    }
    return 1;
}

int tslam_test_potrf_delay(int spins) {
    if (spins < 0 || spins > 100000) return fail(TSLAM_EINVAL, "spins must be in [0, 100000]");
    pose_graph_test_delay(spins);
    return TSLAM_OK;
}

int tslam_pose_graph(tslam_handle* h, int n_nodes, double* world_T_node, int n_edges, const int32_t* edges,
                     const double* meas, const double* info, int iters, double* cost) {
    int64_t id = 0;
    int rc = tslam_loop_job_pose_graph(h, n_nodes, world_T_node, n_edges, edges, meas, info, iters, &id);
    if (rc != TSLAM_OK) return rc;
    rc = tslam_loop_job_poll(h, id, 1, nullptr, nullptr, nullptr, nullptr, world_T_node, cost);
    return rc < 0 ? rc : TSLAM_OK;
}

int tslam_ba_imu_factor(tslam_handle* h, int pair, int64_t frame, const double* M, double weight) {
    if (!h || !M || pair < 0 || pair >= h->P) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    // non-finite inputs would poison the whole window's Schur system (k_ba_solve adds them to S, b)
    if (!(weight >= 0.0) || !std::isfinite(weight) || frame < 0)
        return fail(TSLAM_EINVAL, "weight must be finite and >= 0, frame >= 0");
    for (int e = 0; e < 9; ++e)
        if (!std::isfinite(M[e])) return fail(TSLAM_EINVAL, "rotation M must be finite");
    std::array<double, 10> f{};
    for (int e = 0; e < 9; ++e) f[e] = M[e];
    f[9] = weight;
    h->ba_imu[{pair, frame}] = f;
    return TSLAM_OK;
}

// A rig's inertial factors act on its body window (pair = n_pairs); a stereo pair's on its own.
static int ine_pair_check(tslam_handle* h, int pair) {
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    if (ba_rig(h) ? pair != h->P : (pair < 0 || pair >= h->P))
        return fail(TSLAM_EINVAL, ba_rig(h) ? "a rig's inertial factors go to its body window (pair = n_pairs)"
                                            : "bad pair");
    return TSLAM_OK;
}

int tslam_ba_inertial(tslam_handle* h, int pair, const double* gravity, const double* ba_prior, double ba_weight,
                      const double* bg_prior, double bg_weight) {
    if (!h || !gravity || !ba_prior || !bg_prior) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (int rc = ine_pair_check(h, pair); rc != TSLAM_OK) return rc;
    if (!(ba_weight >= 0.0) || !std::isfinite(ba_weight) || !(bg_weight >= 0.0) || !std::isfinite(bg_weight))
        return fail(TSLAM_EINVAL, "bias weights must be finite and >= 0");
    for (int e = 0; e < 3; ++e)
        if (!std::isfinite(gravity[e]) || !std::isfinite(ba_prior[e]) || !std::isfinite(bg_prior[e]))
            return fail(TSLAM_EINVAL, "non-finite input");
    auto& f = h->ba_icfg[pair];
    for (int e = 0; e < 3; ++e) {
        f[e] = gravity[e];
        f[3 + e] = ba_prior[e];
        f[7 + e] = bg_prior[e];
    }
    f[6] = ba_weight;
    f[10] = bg_weight;
    return TSLAM_OK;
}

int tslam_ba_inertial_factor(tslam_handle* h, int pair, int64_t frame, const double* record, const double* v0) {
    if (!h || !record || !v0 || frame < 0) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (int rc = ine_pair_check(h, pair); rc != TSLAM_OK) return rc;
    std::array<double, TS_BA_INE + 3> f{};
    for (int e = 0; e < TS_BA_INE; ++e) {
        if (!std::isfinite(record[e])) return fail(TSLAM_EINVAL, "non-finite factor record");
        f[e] = record[e];
    }
    if (!(f[27] > 0.0)) return fail(TSLAM_EINVAL, "dt must be > 0");
    for (int e : {28, 29, 30, 31, 71})
        if (!(f[e] >= 0.0)) return fail(TSLAM_EINVAL, "weights must be >= 0");
    for (int e = 0; e < 3; ++e) {
        if (!std::isfinite(v0[e])) return fail(TSLAM_EINVAL, "non-finite velocity");
        f[TS_BA_INE + e] = v0[e];
    }
    h->ba_ine[{pair, frame}] = f;
    return TSLAM_OK;
}

int tslam_ba_read_inertial(tslam_handle* h, int pair, double* velocity, double* bias) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (int rc = ine_pair_check(h, pair); rc != TSLAM_OK) return rc;
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    const size_t W = h->prm.ba_window;
    if (velocity) HIPCHK(hipMemcpy(velocity, h->ba.vel + pair * W * 3, 8 * W * 3, hipMemcpyDeviceToHost));
    if (bias) HIPCHK(hipMemcpy(bias, h->ba.bias + pair * W * 6, 8 * W * 6, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_ba_read(tslam_handle* h, int pair, int64_t* frames, double* cam_T_world, int32_t* landmark,
                  double* points, double* obs_uvd, int32_t* counts) {
    if (!h || pair < 0 || pair > h->P || (pair == h->P && !ba_rig(h))) return fail(TSLAM_EINVAL, "bad handle or pair");
    BA_FLUSH(h);
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    const size_t W = h->prm.ba_window, K = h->g.K, WK = W * K;
    const BaStore& b = h->ba;
    if (frames)
        for (size_t s = 0; s < W; ++s) frames[s] = h->ba_frame[s];
    if (pair == h->P) {   // the rig's body window: body_T_world per slot and the joint counts only
        if (cam_T_world) HIPCHK(hipMemcpy(cam_T_world, b.T + pair * W * 16, 8 * W * 16, hipMemcpyDeviceToHost));
        if (counts) HIPCHK(hipMemcpy(counts, b.counts + 4 * pair, 4 * 4, hipMemcpyDeviceToHost));
        if (landmark) std::fill(landmark, landmark + WK, -1);
        if (points) std::fill(points, points + WK * 3, 0.0);
        if (obs_uvd) std::fill(obs_uvd, obs_uvd + 3 * WK, std::numeric_limits<double>::quiet_NaN());
        return TSLAM_OK;
    }
    if (cam_T_world) HIPCHK(hipMemcpy(cam_T_world, b.T + pair * W * 16, 8 * W * 16, hipMemcpyDeviceToHost));
    if (landmark) HIPCHK(hipMemcpy(landmark, b.lm + pair * WK, 4 * WK, hipMemcpyDeviceToHost));
    if (points) HIPCHK(hipMemcpy(points, b.X + pair * WK * 3, 8 * WK * 3, hipMemcpyDeviceToHost));
    if (obs_uvd) {
        HIPCHK(hipMemcpy(obs_uvd, b.u + pair * WK, 8 * WK, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(obs_uvd + WK, b.v + pair * WK, 8 * WK, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(obs_uvd + 2 * WK, b.d + pair * WK, 8 * WK, hipMemcpyDeviceToHost));
    }
    if (counts) HIPCHK(hipMemcpy(counts, b.counts + 4 * pair, 4 * 4, hipMemcpyDeviceToHost));
    return TSLAM_OK;
}

int tslam_ba_replay_schur(tslam_handle* h, int pair, int reps, void* stream, double* us_per_launch,
                          double* flops_per_launch) {
    if (!h || pair < 0 || pair >= h->P || reps < 1) return fail(TSLAM_EINVAL, "bad argument");
    BA_FLUSH(h);
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    if ((int)h->ba_solved.size() <= pair) return fail(TSLAM_ESTATE, "no window solved yet");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const double zero = 0.0;
    HIPCHK(hipMemcpy(h->ba.flops, &zero, sizeof(double), hipMemcpyHostToDevice));
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    const BatchCtx c = make_ctx(h);
    HIPCHK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch_ba_schur(c, h->ba_solved[pair], s);
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    double fl = 0.0;
    HIPCHK(hipMemcpy(&fl, h->ba.flops, sizeof(double), hipMemcpyDeviceToHost));
    if (us_per_launch) *us_per_launch = 1e3 * ms / reps;
    if (flops_per_launch) *flops_per_launch = fl / reps;
    return TSLAM_OK;
}

int tslam_ba_defer(tslam_handle* h, int defer) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    h->ba_defer = defer != 0;
    return TSLAM_OK;
}

int tslam_ba_graph(tslam_handle* h, int enable) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    h->ba_graph = enable != 0;
    return TSLAM_OK;
}

int tslam_ba_split_solve(tslam_handle* h, int split) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    h->ba_split = split != 0;
    return TSLAM_OK;
}

int tslam_ba_profile(tslam_handle* h, int max_launches, double* schur_ms, int64_t* schur_launches, double* schur_flops) {
    if (!h) return fail(TSLAM_EINVAL, "null handle");
    BA_FLUSH(h);
    if (!h->prm.ba_window) return fail(TSLAM_ESTATE, "local BA is off (ba_window = 0)");
    int rc = tslam_sync(h);
    if (rc != TSLAM_OK) return rc;
    BaTiming& t = h->ba_timing;
    double ms = 0.0;
    for (int i = 0; i < t.used; ++i) {
        float e = 0.0f;
        HIPCHK(hipEventElapsedTime(&e, t.ev[2 * i], t.ev[2 * i + 1]));
        ms += e;
    }
    double fl = 0.0;
    HIPCHK(hipMemcpy(&fl, h->ba.flops, sizeof(double), hipMemcpyDeviceToHost));
    if (schur_ms) *schur_ms = ms;
    if (schur_launches) *schur_launches = t.used;
    if (schur_flops) *schur_flops = t.ev ? fl : 0.0;
    // restart: (re)arm with room for max_launches timed launches, or disarm with 0
    const double zero = 0.0;
    HIPCHK(hipMemcpy(h->ba.flops, &zero, sizeof(double), hipMemcpyHostToDevice));
    t.used = 0;
    if (max_launches < 0) return fail(TSLAM_EINVAL, "max_launches must be >= 0");
    if ((size_t)max_launches * 2 > h->ba_events.size()) {
        while (h->ba_events.size() < (size_t)max_launches * 2) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            h->ba_events.push_back(e);
        }
    }
    t.ev = max_launches ? h->ba_events.data() : nullptr;
    t.cap = max_launches;
    return TSLAM_OK;
}

}  // extern "C"
