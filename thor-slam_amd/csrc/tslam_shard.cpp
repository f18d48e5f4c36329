// tslam_shard.cpp — the library's own driver of a sharded rig (one camera stream per
// GPU; replaces cuVSLAM's multicam mode, launch/thor_visual_slam.launch.py:49,81).
//
// A driver owns, per local rank, the exchange buffers (two sets, by batch parity), three streams and
// the events between them, and runs one batch of every local rank through the stages of a sharded
// handle (tslam_set_shard) with the exchanges in between:
//
//   stereo rig                                         camera-sharded RGB-D rig
//   x : raw images of the frames each peer solves ──┐   f : RECTIFY .. DESCRIBE (own cameras)
//   f : RECTIFY, DETECT, DESCRIBE, pack streams      │   b : MATCH, POSE (own cameras, whole batch),
//   x : ── exchange 1 (raw images, stream blocks) ◄──┘       pack pair blocks per peer range
//   b : import raw + unpack streams, MATCH, POSE(+rig)  b : ── exchange 1 (pair blocks)
//                                                       b : unpack pairs, KERNEL_RIG (own range)
//   b : pack pose records ── exchange 2 (all-gather) ── unpack, CHAIN  (both)
//
// f = front stream (high priority), x = exchange stream, b = back stream.  Batch s's raw exchange
// overlaps its front end and batch s+1's front end overlaps batch s's back end; a parity's receive
// buffers are reused once the imports of batch s-2 are done (event), its send buffers once the
// collectives that read them are.  Nothing here synchronises the host.
//
// Transports: RCCL (ncclSend / ncclRecv / ncclAllGather over xGMI; two communicators per rank so
// the pose all-gather of batch s, on the back stream, never shares a communicator with batch s+1's
// exchange on the exchange stream), created per process (tslam_comm_init: one local rank) or for
// all devices of one process (tslam_group_create: ncclCommInitAll); or COPY (device-to-device
// copies pushed on the sender's stream: a group of ranks in one process, also several on one device
// — the same packing and ordering as RCCL, used to test world > 1 on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "tslam_internal.h"

#define SHCHK(expr)                                                                                            \
    do {                                                                                                       \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            return tslam_internal_fail(TSLAM_EHIP, (std::string(#expr) + ": " + hipGetErrorString(e__)).c_str()); \
    } while (0)
#define NCCLCHK(expr)                                                                                          \
    do {                                                                                                       \
        ncclResult_t r__ = (expr);                                                                             \
        if (r__ != ncclSuccess)                                                                                \
            return tslam_internal_fail(TSLAM_EHIP, (std::string(#expr) + ": " + ncclGetErrorString(r__)).c_str()); \
    } while (0)
#define RC(expr)                          \
    do {                                  \
        const int rc__ = (expr);          \
        if (rc__ != TSLAM_OK) return rc__; \
    } while (0)

namespace {
struct Rank {
    tslam_handle* h = nullptr;
    int rank = 0, device = 0;
    ncclComm_t comm_x = nullptr, comm_p = nullptr;
    hipStream_t fs = nullptr, xs = nullptr, bs = nullptr;
    hipEvent_t ev_in = nullptr, ev_front = nullptr, ev_x = nullptr, ev_push = nullptr, ev_done = nullptr;
    hipEvent_t consumed[2] = {nullptr, nullptr};   // this parity's receive buffers were read
    bool consumed_armed[2] = {false, false};
    bool done_armed = false;
    uint8_t* raw_send[2] = {nullptr, nullptr};
    uint8_t* raw_recv[2] = {nullptr, nullptr};
    uint8_t* feat_send[2] = {nullptr, nullptr};    // stream blocks (stereo) or pair blocks (RGB-D)
    uint8_t* feat_recv[2] = {nullptr, nullptr};
    uint8_t* pose_send[2] = {nullptr, nullptr};
    uint8_t* pose_recv[2] = {nullptr, nullptr};
    uint8_t* prev_raw = nullptr;   // the previous batch's last frame of this rank's cameras
    std::vector<void*> allocs;
};

enum Which { RAW = 0, FEAT = 1, POSE = 2 };
}  // namespace

struct tslam_shard_driver {
    int world = 1, transport = TSLAM_TRANSPORT_RCCL;
    bool rgbd = false, rig = false;
    int S = 0, B = 0;                    // cameras per rank, max_batch
    int n = 0, fpr = 0, nr = 0;          // this batch: frames, frames per rank, frames sent per peer (stereo)
    size_t img = 0, rec = 0, sblk = 0, pblk = 0;   // bytes: image, pose record, stream block, pair block
    size_t raw_q = 0, feat_q = 0;        // this batch: bytes per peer (raw images, stream / pair blocks)
    int64_t batches = 0;
    std::vector<Rank> ranks;   // local ranks: all of a group, one after tslam_comm_init
};

static void destroy_driver(tslam_shard_driver* d) {
    if (!d) return;
    for (Rank& r : d->ranks) {
        (void)hipSetDevice(r.device);
        (void)hipDeviceSynchronize();
        if (r.comm_p) (void)ncclCommDestroy(r.comm_p);
        if (r.comm_x) (void)ncclCommDestroy(r.comm_x);
        for (hipEvent_t e : {r.ev_in, r.ev_front, r.ev_x, r.ev_push, r.ev_done, r.consumed[0], r.consumed[1]})
            if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : {r.fs, r.xs, r.bs})
            if (s) (void)hipStreamDestroy(s);
        for (void* p : r.allocs) (void)hipFree(p);
        r.allocs.clear();
    }
    delete d;
}

extern "C" void tslam_internal_driver_destroy(tslam_shard_driver* d) { destroy_driver(d); }

static int alloc(Rank& r, uint8_t** p, size_t bytes) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    if (e != hipSuccess) return tslam_internal_fail(TSLAM_ENOMEM, (std::string("hipMalloc: ") + hipGetErrorString(e)).c_str());
    r.allocs.push_back(q);
    *p = (uint8_t*)q;
    SHCHK(hipMemset(q, 0, bytes ? bytes : 16));
    return TSLAM_OK;
}

// Geometry of the driver from its ranks' handles (all the same rig, sharded by tslam_set_shard).
static int plan(tslam_shard_driver* d, tslam_handle* h, int world) {
    tslam_handle_info in{};
    RC(tslam_internal_info(h, &in));
    if (in.ba) return tslam_internal_fail(TSLAM_EINVAL, "sharding covers rigs without local BA");
    if (in.C % world || in.B % world)
        return tslam_internal_fail(TSLAM_EINVAL, "cameras and max_batch must divide by world");
    d->world = world;
    d->rgbd = in.rgbd != 0;
    d->rig = in.rig != 0;
    d->S = in.C / world;
    d->B = in.B;
    d->img = (size_t)in.W * in.H;
    d->rec = (size_t)in.pose_record;
    d->sblk = (size_t)in.stream_block;
    d->pblk = (size_t)in.pair_block;
    return TSLAM_OK;
}

// Per-batch geometry of n frames (n % world == 0, n <= max_batch): the buffers are sized for
// max_batch, a shorter batch uses the front of each per-peer slot.
static void geom(tslam_shard_driver* d, int n) {
    d->n = n;
    d->fpr = n / d->world;
    d->nr = d->fpr + 1;
    if (d->rgbd) {
        d->raw_q = 0;
        d->feat_q = (size_t)d->fpr * d->S * d->pblk;   // my cameras' pair blocks of a peer's range
    } else {
        d->raw_q = (size_t)d->nr * d->S * d->img;        // frames lo-1 .. hi-1 of a peer's range
        d->feat_q = (size_t)d->nr * d->S * d->sblk;
    }
}

static int setup_rank(tslam_shard_driver* d, Rank& r) {
    tslam_handle_info in{};
    RC(tslam_internal_info(r.h, &in));
    r.device = in.device;
    SHCHK(hipSetDevice(r.device));
    int lo = 0, hi = 0;
    SHCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    SHCHK(hipStreamCreateWithPriority(&r.fs, hipStreamNonBlocking, hi));   // the front end is the critical path
    SHCHK(hipStreamCreateWithFlags(&r.xs, hipStreamNonBlocking));
    SHCHK(hipStreamCreateWithFlags(&r.bs, hipStreamNonBlocking));
    for (hipEvent_t* e : {&r.ev_in, &r.ev_front, &r.ev_x, &r.ev_push, &r.ev_done, &r.consumed[0], &r.consumed[1]})
        SHCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    const size_t N = d->world;
    geom(d, d->B);   // allocation sizes: a full batch
    for (int k = 0; k < 2; ++k) {
        if (!d->rgbd) {
            RC(alloc(r, &r.raw_send[k], N * d->raw_q));
            RC(alloc(r, &r.raw_recv[k], N * d->raw_q));
        }
        RC(alloc(r, &r.feat_send[k], N * d->feat_q));
        RC(alloc(r, &r.feat_recv[k], N * d->feat_q));
        RC(alloc(r, &r.pose_send[k], (size_t)d->fpr * d->rec));
        RC(alloc(r, &r.pose_recv[k], N * d->fpr * d->rec));
    }
    if (!d->rgbd) RC(alloc(r, &r.prev_raw, (size_t)d->S * d->img));
    SHCHK(hipDeviceSynchronize());   // the zeroing (null stream) lands before the rank's streams use them
    return TSLAM_OK;
}

// The stream an exchange runs on (sender and receiver side): stereo raw images and stream blocks
// on the exchange stream, pair blocks and pose records on the back stream.
static hipStream_t xstream(const tslam_shard_driver* d, const Rank& r, Which w) {
    return (w == POSE || d->rgbd) ? r.bs : r.xs;
}

static int exchange(tslam_shard_driver* d, Which w, int k) {
    const int N = d->world;
    if (d->transport == TSLAM_TRANSPORT_RCCL) {
        NCCLCHK(ncclGroupStart());
        for (Rank& r : d->ranks) {
            hipStream_t s = xstream(d, r, w);
            if (w == POSE) {
                NCCLCHK(ncclAllGather(r.pose_send[k], r.pose_recv[k], (size_t)d->fpr * d->rec, ncclUint8, r.comm_p, s));
                continue;
            }
            uint8_t* snd = w == RAW ? r.raw_send[k] : r.feat_send[k];
            uint8_t* rcv = w == RAW ? r.raw_recv[k] : r.feat_recv[k];
            const size_t u = w == RAW ? d->raw_q : d->feat_q;
            for (int q = 0; q < N; ++q) {
                if (q == r.rank) continue;
                NCCLCHK(ncclSend(snd + q * u, u, ncclUint8, q, r.comm_x, s));
                NCCLCHK(ncclRecv(rcv + q * u, u, ncclUint8, q, r.comm_x, s));
            }
        }
        NCCLCHK(ncclGroupEnd());
        return TSLAM_OK;
    }
    // COPY: each sender pushes into its peers' receive buffers on its own exchange-side stream,
    // once the peer has consumed the previous use of that parity; the receivers wait for every push
    for (Rank& src : d->ranks) {
        SHCHK(hipSetDevice(src.device));
        hipStream_t s = xstream(d, src, w);
        for (Rank& dst : d->ranks) {
            if (w == POSE) {
                if (dst.done_armed && &dst != &src) SHCHK(hipStreamWaitEvent(s, dst.ev_done, 0));
                SHCHK(hipMemcpyAsync(dst.pose_recv[k] + (size_t)src.rank * d->fpr * d->rec, src.pose_send[k],
                                     (size_t)d->fpr * d->rec, hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (&dst == &src) continue;
            if (dst.consumed_armed[k]) SHCHK(hipStreamWaitEvent(s, dst.consumed[k], 0));
            const size_t u = w == RAW ? d->raw_q : d->feat_q;
            const uint8_t* snd = (w == RAW ? src.raw_send[k] : src.feat_send[k]) + (size_t)dst.rank * u;
            uint8_t* rcv = (w == RAW ? dst.raw_recv[k] : dst.feat_recv[k]) + (size_t)src.rank * u;
            SHCHK(hipMemcpyAsync(rcv, snd, u, hipMemcpyDeviceToDevice, s));
        }
        SHCHK(hipEventRecord(src.ev_push, s));
    }
    for (Rank& dst : d->ranks) {
        SHCHK(hipSetDevice(dst.device));
        hipStream_t s = xstream(d, dst, w);
        for (Rank& src : d->ranks)
            if (&src != &dst) SHCHK(hipStreamWaitEvent(s, src.ev_push, 0));
    }
    return TSLAM_OK;
}

// Raw images of this rank's cameras for every peer: its frames lo-1 .. hi-1 (frame -1 = the last
// frame of the previous batch), one gather launch on the exchange stream; then this batch's last
// frame becomes prev_raw.
static int stage_raw(tslam_shard_driver* d, Rank& r, const uint8_t* images, int k) {
    const size_t frame = (size_t)d->S * d->img;
    if (d->world > 1) RC(tslam_stage_raw_peers(r.h, r.prev_raw, r.raw_send[k], r.xs));
    SHCHK(hipMemcpyAsync(r.prev_raw, images + (size_t)(d->n - 1) * frame, frame, hipMemcpyDeviceToDevice, r.xs));
    return TSLAM_OK;
}

static int submit(tslam_shard_driver* d, const uint8_t* const* images, int n, void* const* streams) {
    if (n < d->world || n > d->B || n % d->world)
        return tslam_internal_fail(TSLAM_EINVAL, "a sharded batch needs world <= n_frames <= max_batch, n_frames % world == 0");
    geom(d, n);
    const int k = (int)(d->batches & 1), N = d->world, S = d->S;
    const int front[3] = {TSLAM_STAGE_RECTIFY, TSLAM_STAGE_DETECT, TSLAM_STAGE_DESCRIBE};
    for (size_t i = 0; i < d->ranks.size(); ++i) {   // inputs, buffer reuse, raw images out
        Rank& r = d->ranks[i];
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_in, streams ? (hipStream_t)streams[i] : nullptr));
        for (hipStream_t s : {r.fs, r.xs, r.bs}) SHCHK(hipStreamWaitEvent(s, r.ev_in, 0));
        if (r.consumed_armed[k])
            for (hipStream_t s : {r.fs, r.xs}) SHCHK(hipStreamWaitEvent(s, r.consumed[k], 0));
        RC(tslam_begin_batch(r.h, images[i], n));
        if (!d->rgbd) RC(stage_raw(d, r, images[i], k));
    }
    if (!d->rgbd) RC(exchange(d, RAW, k));
    for (Rank& r : d->ranks) {   // front end of the rank's cameras (+ its stream blocks per peer)
        for (int st : front) RC(tslam_run_stage(r.h, st, r.fs));
        if (d->rgbd) continue;
        if (N > 1) RC(tslam_pack_streams_peers(r.h, r.feat_send[k], r.fs));   // every peer's frames, one launch
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_front, r.fs));
        SHCHK(hipStreamWaitEvent(r.xs, r.ev_front, 0));
    }
    if (!d->rgbd) RC(exchange(d, FEAT, k));
    for (Rank& r : d->ranks) {   // back end
        if (!d->rgbd) {
            // the other cameras of frames lo-1 .. hi-1 of this rank's range into the ring
            SHCHK(hipSetDevice(r.device));
            SHCHK(hipEventRecord(r.ev_x, r.xs));
            SHCHK(hipStreamWaitEvent(r.bs, r.ev_x, 0));
            if (N > 1) RC(tslam_import_peers(r.h, r.raw_recv[k], r.feat_recv[k], r.bs));
            SHCHK(hipEventRecord(r.consumed[k], r.bs));
            r.consumed_armed[k] = true;
        }
        RC(tslam_run_stage(r.h, TSLAM_STAGE_MATCH, r.bs));
        RC(tslam_run_stage(r.h, TSLAM_STAGE_POSE, r.bs));
        if (d->rgbd)   // this rank's cameras over every peer's frame range
            for (int q = 0; q < N; ++q)
                if (q != r.rank)
                    RC(tslam_pack_pairs(r.h, q * d->fpr, d->fpr, r.rank * S, (r.rank + 1) * S,
                                        r.feat_send[k] + (size_t)q * d->feat_q, r.bs));
    }
    if (d->rgbd) {
        RC(exchange(d, FEAT, k));
        for (Rank& r : d->ranks) {
            for (int q = 0; q < N; ++q)
                if (q != r.rank)
                    RC(tslam_unpack_pairs(r.h, r.rank * d->fpr, d->fpr, q * S, (q + 1) * S,
                                          r.feat_recv[k] + (size_t)q * d->feat_q, r.bs));
            SHCHK(hipSetDevice(r.device));
            SHCHK(hipEventRecord(r.consumed[k], r.bs));
            r.consumed_armed[k] = true;
            if (d->rig) RC(tslam_run_stage(r.h, TSLAM_KERNEL_RIG, r.bs));
        }
    }
    for (Rank& r : d->ranks) RC(tslam_pack_poses(r.h, r.pose_send[k], r.bs));
    RC(exchange(d, POSE, k));
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        Rank& r = d->ranks[i];
        RC(tslam_unpack_poses(r.h, r.pose_recv[k], r.bs));
        RC(tslam_run_stage(r.h, TSLAM_KERNEL_CHAIN, r.bs));
        RC(tslam_end_batch(r.h));
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_done, r.bs));
        r.done_armed = true;
        // the caller's stream orders after the batch (results in stream order)
        SHCHK(hipStreamWaitEvent(streams ? (hipStream_t)streams[i] : nullptr, r.ev_done, 0));
    }
    d->batches += 1;
    return TSLAM_OK;
}

extern "C" {

int tslam_comm_unique_id(void* id128) {
    if (!id128) return tslam_internal_fail(TSLAM_EINVAL, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(id128, &id, sizeof(id));
    return TSLAM_OK;
}

int tslam_comm_init(tslam_handle* h, const void* id128, int rank, int world) {
    if (!h || !id128) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    if (tslam_internal_driver(h)) return tslam_internal_fail(TSLAM_ESTATE, "communicator already set");
    if (world < 1 || rank < 0 || rank >= world) return tslam_internal_fail(TSLAM_EINVAL, "need 0 <= rank < world");
    auto* d = new tslam_shard_driver();
    int rc = plan(d, h, world);
    if (rc == TSLAM_OK) rc = tslam_set_shard(h, rank * d->S, (rank + 1) * d->S, rank, world);
    if (rc != TSLAM_OK) {
        delete d;
        return rc;
    }
    d->transport = TSLAM_TRANSPORT_RCCL;
    d->ranks.resize(1);
    Rank& r = d->ranks[0];
    r.h = h;
    r.rank = rank;
    rc = setup_rank(d, r);
    if (rc == TSLAM_OK) {
        ncclUniqueId id;
        memcpy(&id, id128, sizeof(id));
        ncclResult_t nr = ncclCommInitRank(&r.comm_x, world, id, rank);
        // the pose all-gather's own communicator (same ranks)
        if (nr == ncclSuccess) nr = ncclCommSplit(r.comm_x, 0, rank, &r.comm_p, nullptr);
        if (nr != ncclSuccess) rc = tslam_internal_fail(TSLAM_EHIP, (std::string("RCCL communicator: ") + ncclGetErrorString(nr)).c_str());
    }
    if (rc == TSLAM_OK) rc = tslam_internal_attach_driver(h, d, true);
    if (rc != TSLAM_OK) {
        (void)tslam_set_shard(h, 0, (int)(d->S * world), 0, 1);
        destroy_driver(d);
    }
    return rc;
}

int tslam_submit_sharded(tslam_handle* h, const uint8_t* images, void* stream) {
    if (!h || !images) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    tslam_shard_driver* d = tslam_internal_driver(h);
    if (!d || d->ranks.size() != 1) return tslam_internal_fail(TSLAM_ESTATE, "tslam_comm_init first");
    void* streams[1] = {stream};
    return submit(d, &images, d->B, streams);
}

struct tslam_group {
    tslam_shard_driver* d = nullptr;
};

int tslam_group_create(tslam_handle* const* handles, int n, int transport, tslam_group** out) {
    if (!handles || n < 1 || !out) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    if (transport != TSLAM_TRANSPORT_RCCL && transport != TSLAM_TRANSPORT_COPY)
        return tslam_internal_fail(TSLAM_EINVAL, "transport must be TSLAM_TRANSPORT_RCCL or TSLAM_TRANSPORT_COPY");
    tslam_handle_info in0{};
    RC(tslam_internal_info(handles[0], &in0));
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        tslam_handle_info in{};
        if (!handles[i]) return tslam_internal_fail(TSLAM_EINVAL, "null handle");
        RC(tslam_internal_info(handles[i], &in));
        if (in.C != in0.C || in.P != in0.P || in.B != in0.B || in.W != in0.W || in.H != in0.H || in.rgbd != in0.rgbd ||
            in.rig != in0.rig)
            return tslam_internal_fail(TSLAM_EINVAL, "a group's handles must describe the same rig and batch");
        if (tslam_internal_driver(handles[i])) return tslam_internal_fail(TSLAM_ESTATE, "handle already driven");
        devs[i] = in.device;
        for (int j = 0; j < i; ++j)
            if (transport == TSLAM_TRANSPORT_RCCL && devs[j] == devs[i])
                return tslam_internal_fail(TSLAM_EINVAL, "an RCCL group needs one device per handle (COPY allows sharing)");
    }
    auto* d = new tslam_shard_driver();
    int rc = plan(d, handles[0], n);
    d->transport = transport;
    d->ranks.resize(n);
    for (int i = 0; i < n && rc == TSLAM_OK; ++i) {
        d->ranks[i].h = handles[i];
        d->ranks[i].rank = i;
        rc = tslam_set_shard(handles[i], i * d->S, (i + 1) * d->S, i, n);
        if (rc == TSLAM_OK) rc = setup_rank(d, d->ranks[i]);
    }
    if (rc == TSLAM_OK && transport == TSLAM_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> cx(n), cp(n);
        ncclResult_t nr = ncclCommInitAll(cx.data(), n, devs.data());
        if (nr == ncclSuccess) nr = ncclCommInitAll(cp.data(), n, devs.data());
        if (nr != ncclSuccess) {
            rc = tslam_internal_fail(TSLAM_EHIP, (std::string("ncclCommInitAll: ") + ncclGetErrorString(nr)).c_str());
        } else {
            for (int i = 0; i < n; ++i) {
                d->ranks[i].comm_x = cx[i];
                d->ranks[i].comm_p = cp[i];
            }
        }
    }
    for (int i = 0; i < n && rc == TSLAM_OK; ++i) rc = tslam_internal_attach_driver(handles[i], d, false);
    if (rc != TSLAM_OK) {
        for (int i = 0; i < n; ++i) {
            (void)tslam_internal_attach_driver(handles[i], nullptr, false);
            (void)tslam_set_shard(handles[i], 0, in0.C, 0, 1);
        }
        destroy_driver(d);
        return rc;
    }
    *out = new tslam_group{d};
    return TSLAM_OK;
}

int tslam_group_submit(tslam_group* g, const uint8_t* const* images, int n_frames, void* const* streams) {
    if (!g || !g->d || !images) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    for (size_t i = 0; i < g->d->ranks.size(); ++i)
        if (!images[i]) return tslam_internal_fail(TSLAM_EINVAL, "null images");
    return submit(g->d, images, n_frames, streams);
}

int tslam_group_destroy(tslam_group* g) {
    if (!g) return TSLAM_OK;
    if (g->d) {
        const int C = g->d->S * g->d->world;
        for (Rank& r : g->d->ranks) {
            (void)tslam_internal_attach_driver(r.h, nullptr, false);
            (void)tslam_set_shard(r.h, 0, C, 0, 1);
        }
        destroy_driver(g->d);
    }
    delete g;
    return TSLAM_OK;
}

}  // extern "C"
