"""Sharded rig: one camera stream per GPU (BASELINE.json ``north_star``).

The reference hands a multi-camera rig to cuVSLAM's multicam mode as one process
(``launch/thor_visual_slam.launch.py:49,81``; the rig is ``RigCalibration.get_world_extrinsics``,
``thor_slam/camera/rig.py:35-70``, in the camera order of ``IsaacRosAdapter._extract_cameras``,
``thor_slam/slam/adapters/isaac_ros.py:138-157``).  Here the rig is spread over ``world`` ranks,
one process per GPU:

* **streams**: rank r owns cameras ``[r*S, (r+1)*S)`` (S = cameras / world; S = 1 is one camera
  stream per GPU) and runs the front end (rectify, pyramid, FAST/NMS/top-K, orientation +
  rBRIEF) of those cameras for every frame of a batch;
* **frames**: rank r owns batch frames ``[r*B/world, (r+1)*B/world)`` and runs the back end of
  every stereo pair for them (stereo + temporal Hamming matching with sub-pixel refinement,
  P3P-RANSAC + Gauss-Newton) and the rig pose (generalised PnP over all pairs' correspondences);
* **exchange 1** (RCCL all-to-all): each rank sends every other rank the frames that rank solves
  (its range plus the frame before, whose stereo disparities the range's first frame
  triangulates from): the raw images of its cameras and their stream blocks (keypoints,
  y-sorted records, descriptors, row index; ``tslam_pack_streams``);
* **exchange 2** (RCCL all-gather): the per-frame pose records (per-pair and rig poses), after
  which every rank chains the whole batch identically.

Every rank ends the batch with exactly the poses an unsharded handle fed all cameras produces
(same kernels on the same data; ``tests/test_gpu_shard.py``).  An all-gather of the stream
blocks (``exchange="allgather"``) is the literal reading of ``north_star`` and is kept as an
option: it sends every frame to every rank, ``world`` times the bytes of the all-to-all.

An RGB-D rig (each "pair" is one colour camera with its aligned depth, ``HipSlamConfig.rgbd``)
shards by camera only and moves no image: every rank tracks its own cameras over the whole batch
(front end, temporal match + depth lookup, P3P-RANSAC + Gauss-Newton), then **exchange 1** is an
all-to-all of *pair blocks* (per frame and camera: pose record, stats and the 3D-2D
correspondences, ``tslam_pack_pairs``) so that each rank solves the rig pose of its frame range
over all cameras; exchange 2 and the chain are as above.

Three drivers share :class:`RankShard` (one rank's handle, buffers and phases):
:class:`LocalShardedRig` (all ranks in one process on one device: tests and rehearsal),
:class:`DistShardedRig` (one rank of a ``torch.distributed`` job, backend ``nccl`` = RCCL, or
``gloo`` staging through the host).
"""

from __future__ import annotations

from dataclasses import dataclass

from ._lib import Handle


@dataclass(frozen=True)
class ShardPlan:
    """Which cameras and which batch frames each of ``world`` ranks owns."""

    n_cams: int
    world: int
    batch: int

    def __post_init__(self) -> None:
        if self.world < 1 or self.n_cams % self.world:
            raise ValueError(f"{self.n_cams} cameras do not split over {self.world} ranks")
        if self.batch % self.world:
            raise ValueError(f"batch {self.batch} is not a multiple of world {self.world}")

    @property
    def streams_per_rank(self) -> int:
        return self.n_cams // self.world

    @property
    def frames_per_rank(self) -> int:
        return self.batch // self.world

    @property
    def recv_frames(self) -> int:
        """Frames of another rank's cameras a rank receives per batch: its range + the frame before."""
        return self.frames_per_rank + 1

    def cams(self, rank: int) -> tuple[int, int]:
        s = self.streams_per_rank
        return rank * s, (rank + 1) * s

    def frames(self, rank: int) -> tuple[int, int]:
        f = self.frames_per_rank
        return rank * f, (rank + 1) * f

    def sent_frames(self, rank: int) -> tuple[int, int]:
        """Batch frames [a, b) of every camera that rank ``rank`` needs from the others: its range
        and the frame before (a = -1: the previous batch's last frame)."""
        lo, hi = self.frames(rank)
        return lo - 1, hi


def _timed(timer, name, fn) -> None:
    if timer is None:
        fn()
        return
    timer.begin(name)
    fn()
    timer.end(name)


class StageTimer:
    """HIP events around each kernel of the phases it is handed, on the torch stream set in
    ``stream`` (the stream those kernels are launched on: torch.cuda.Event only sees that one)."""

    def __init__(self):
        self.stream = None
        self.spans: dict[str, list] = {}
        self._open = None

    def begin(self, name: str) -> None:
        import torch

        e = torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        self._open = e

    def end(self, name: str) -> None:
        import torch

        e = torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        self.spans.setdefault(name, []).append((self._open, e))

    def event(self, stream):
        """A timing event recorded on ``stream`` now (for spans across streams)."""
        import torch

        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def span(self, name: str, e0, e1) -> None:
        self.spans.setdefault(name, []).append((e0, e1))

    def mean_us(self) -> dict[str, float]:
        """Average microseconds per launch of each name (synchronise first)."""
        return {k: sum(a.elapsed_time(b) for a, b in v) * 1e3 / len(v) for k, v in self.spans.items()}


class RankShard:
    """One rank of a sharded rig: its handle (the whole rig's geometry, its own cameras' front
    end, its frame range's back end) and the device buffers of the two exchanges."""

    def __init__(self, rects: list, cfg, plan: ShardPlan, rank: int, base_T_rect: list | None = None,
                 device: int = 0, exchange: str = "alltoall"):
        import torch

        self.torch = torch
        self.plan = plan
        self.rank = rank
        self.exchange = exchange
        self.h = Handle(rects, cfg, max_batch=plan.batch, device=device)
        if base_T_rect is not None and len(rects) > 1:
            self.h.set_rig(base_T_rect)
        self.rig = base_T_rect is not None and len(rects) > 1
        self.rgbd = bool(cfg.rgbd)
        self.cam_lo, self.cam_hi = plan.cams(rank)
        self.h.set_shard(self.cam_lo, self.cam_hi, rank, plan.world)
        self.block, self.record = self.h.exchange_sizes()
        W, H = self.h.width, self.h.height
        S, N, nr = plan.streams_per_rank, plan.world, plan.recv_frames
        self.img_bytes = W * H
        dev = torch.device("cuda", device)
        self.dev = dev
        self.batches = 0
        if self.rgbd:
            # pair blocks: to each peer q, this rank's cameras over q's frame range
            self.pblock = self.h.pair_block_bytes()
            fpr = plan.frames_per_rank
            self.frames_sent = fpr
            self.feat_send = [torch.empty((N, fpr, S, self.pblock), dtype=torch.uint8, device=dev) for _ in range(2)]
            self.feat_recv = [torch.empty((N, fpr, S, self.pblock), dtype=torch.uint8, device=dev) for _ in range(2)]
            self.raw_send = self.raw_recv = None
            self._pose_buffers(torch, dev)
            return
        # per destination q: [nr][S][H*W] raw images and [nr][S][block] stream blocks (the
        # all-gather variant sends all B+1 frames to everyone); two sets by batch parity
        fr = nr if exchange == "alltoall" else plan.batch + 1
        self.frames_sent = fr
        nd = N if exchange == "alltoall" else 1
        self.raw_send = [torch.empty((nd, fr, S, W * H), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.raw_recv = [torch.empty((N, fr, S, W * H), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.feat_send = [torch.empty((nd, fr, S, self.block), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.feat_recv = [torch.empty((N, fr, S, self.block), dtype=torch.uint8, device=dev) for _ in range(2)]
        self._pose_buffers(torch, dev)
        self.prev_raw = torch.zeros((S, W * H), dtype=torch.uint8, device=dev)   # last frame of the previous batch

    def _pose_buffers(self, torch, dev) -> None:
        N, fpr = self.plan.world, self.plan.frames_per_rank
        self.pose_send = [torch.empty((fpr, self.record), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.pose_recv = [torch.empty((N, fpr, self.record), dtype=torch.uint8, device=dev) for _ in range(2)]

    @property
    def g0(self) -> int:
        return self.h.frames_done

    def _first_sent(self, q: int) -> int:
        """Global index of the first frame sent to rank q (its range start - 1)."""
        a = self.plan.sent_frames(q)[0] if self.exchange == "alltoall" else -1
        return self.g0 + a

    # -- phases of one batch (all enqueued on the given streams; nothing synchronises) ----------
    def begin(self, images) -> None:
        """images: device u8 [B][S][H][W] of this rank's cameras."""
        self.images = images
        self.h.begin_batch(images.data_ptr(), self.plan.batch)

    def stage_raw(self, stream) -> None:
        """Raw images of the frames each destination solves -> raw_send (torch copies on `stream`)."""
        torch = self.torch
        k = self.batches % 2
        imgs = self.images.reshape(self.plan.batch, self.plan.streams_per_rank, -1)
        if self.exchange == "alltoall" and self.plan.world > 1:   # every peer's frames, one gather launch
            self.h.stage_raw_peers(self.prev_raw.data_ptr(), self.raw_send[k].data_ptr(), stream.cuda_stream)
            with torch.cuda.stream(stream):
                self.prev_raw.copy_(imgs[-1])
            return
        with torch.cuda.stream(stream):
            dests = range(self.plan.world) if self.exchange == "alltoall" else [0]
            for j, q in enumerate(dests):
                a, b = self.plan.sent_frames(q) if self.exchange == "alltoall" else (-1, self.plan.batch)
                out = self.raw_send[k][j]
                out[0].copy_(self.prev_raw if a < 0 else imgs[a])
                out[1:].copy_(imgs[a + 1:b])
            self.prev_raw.copy_(imgs[-1])

    def front(self, stream: int, timer=None) -> None:
        for k in ("rectify_pyramid", "detect", "select", "describe"):
            _timed(timer, k, lambda: self.h.run_kernel(k, stream))

    def pack_features(self, stream: int) -> None:
        k = self.batches % 2
        if self.exchange == "alltoall" and self.plan.world > 1:
            self.h.pack_streams_peers(self.feat_send[k].data_ptr(), stream)
            return
        dests = range(self.plan.world) if self.exchange == "alltoall" else [0]
        for j, q in enumerate(dests):
            self.h.pack_streams(self._first_sent(q), self.frames_sent, self.cam_lo, self.cam_hi,
                                self.feat_send[k][j].data_ptr(), stream)

    def import_remote(self, stream: int, timer=None) -> None:
        _timed(timer, "import", lambda: self._import_remote(stream))

    def _import_remote(self, stream: int) -> None:
        """The other ranks' cameras of frames lo-1 .. hi-1 into the ring: raw -> rectify +
        pyramid, stream blocks -> keypoints / records / descriptors."""
        k = self.batches % 2
        if self.exchange == "alltoall" and self.plan.world > 1:   # rectify + unpack every peer, two launches
            self.h.import_peers(self.raw_recv[k].data_ptr(), self.feat_recv[k].data_ptr(), stream)
            return
        lo, hi = self.plan.frames(self.rank)
        for q in range(self.plan.world):
            if q == self.rank:
                continue
            c0, c1 = self.plan.cams(q)
            if self.exchange == "alltoall":
                raw, feat, first = self.raw_recv[k][q], self.feat_recv[k][q], self.g0 + lo - 1
            else:   # all-gather: every frame of the batch (+ the one before); take lo-1 .. hi-1
                raw, feat, first = self.raw_recv[k][q][lo:hi + 1], self.feat_recv[k][q][lo:hi + 1], self.g0 + lo - 1
            self.h.import_raw(raw.data_ptr(), first, hi - lo + 1, c0, c1, stream)
            self.h.unpack_streams(first, hi - lo + 1, c0, c1, feat.data_ptr(), stream)

    def back(self, stream: int, timer=None) -> None:
        for k in ("match", "match_refine", "pose"):
            _timed(timer, k, lambda: self.h.run_kernel(k, stream))
        if self.rgbd:   # the rig pose waits for the other cameras' pair blocks
            return
        if self.rig:
            _timed(timer, "rig", lambda: self.h.run_rig(stream))
        self.h.pack_poses(self.pose_send[self.batches % 2].data_ptr(), stream)

    # -- RGB-D: pair blocks (this rank's cameras tracked over the whole batch) ------------------
    def pack_pairs(self, stream: int) -> None:
        k, fpr = self.batches % 2, self.plan.frames_per_rank
        for q in range(self.plan.world):
            if q != self.rank:
                self.h.pack_pairs(q * fpr, fpr, self.cam_lo, self.cam_hi, self.feat_send[k][q].data_ptr(), stream)

    def rig_range(self, stream: int, timer=None) -> None:
        """The other ranks' pair blocks of this rank's frame range in, its rig pose, its pose records out."""
        k, fpr = self.batches % 2, self.plan.frames_per_rank
        for q in range(self.plan.world):
            if q != self.rank:
                c0, c1 = self.plan.cams(q)
                self.h.unpack_pairs(self.rank * fpr, fpr, c0, c1, self.feat_recv[k][q].data_ptr(), stream)
        if self.rig:
            _timed(timer, "rig", lambda: self.h.run_rig(stream))
        self.h.pack_poses(self.pose_send[k].data_ptr(), stream)

    def finish(self, stream: int, timer=None) -> None:
        self.h.unpack_poses(self.pose_recv[self.batches % 2].data_ptr(), stream)
        _timed(timer, "chain", lambda: self.h.run_kernel("chain", stream))
        self.h.end_batch()
        self.batches += 1

    def read(self, n: int | None = None) -> dict:
        n = self.plan.batch if n is None else n
        out = {"pairs": self.h.read_poses(n)}
        if self.rig:
            out["rig"] = self.h.read_rig_poses(n)
        return out

    def close(self) -> None:
        self.h.close()


class LocalShardedRig:
    """Every rank of a sharded rig in one process on one device: the collectives become device
    copies between the ranks' buffers, everything on one stream.  Same handles, kernels and
    buffers as :class:`DistShardedRig`; used by the tests and as a one-GPU rehearsal."""

    def __init__(self, rects: list, cfg, world: int, batch: int, base_T_rect: list | None = None, device: int = 0,
                 exchange: str = "alltoall"):
        import torch

        self.torch = torch
        n_cams = (1 if cfg.rgbd else 2) * len(rects)
        self.plan = ShardPlan(n_cams, world, batch)
        self.ranks = [RankShard(rects, cfg, self.plan, r, base_T_rect, device, exchange) for r in range(world)]
        self.exchange = exchange
        self.rgbd = bool(cfg.rgbd)

    def step(self, images, stream=None, timer: StageTimer | None = None) -> None:
        """images: device u8 [B][C][H][W] (all cameras; RGB-D records [B][C][5HW]); rank r gets its
        cameras' slice.  With ``timer`` (its stream = ``stream``) every phase of every rank is
        timed on the one stream: the kernels by name, ``stage_raw``, ``pack``, ``exchange`` (the
        device copies standing in for the all-to-all), ``import``, ``pose_gather``."""
        torch = self.torch
        st = stream or torch.cuda.current_stream()
        sp = st.cuda_stream
        S = self.plan.streams_per_rank
        parts = [images[:, r * S:(r + 1) * S].contiguous() for r in range(self.plan.world)]
        if self.rgbd:
            self._step_rgbd(parts, st)
            return
        for r, rk in enumerate(self.ranks):
            rk.begin(parts[r])
            _timed(timer, "stage_raw", lambda: rk.stage_raw(st))
            rk.front(sp, timer)
            _timed(timer, "pack", lambda: rk.pack_features(sp))

        def all_to_all():
            with torch.cuda.stream(st):
                for r, rk in enumerate(self.ranks):
                    k = rk.batches % 2
                    for q, src in enumerate(self.ranks):
                        j = r if self.exchange == "alltoall" else 0
                        rk.raw_recv[k][q].copy_(src.raw_send[k][j])
                        rk.feat_recv[k][q].copy_(src.feat_send[k][j])
        _timed(timer, "exchange", all_to_all)
        for rk in self.ranks:
            rk.import_remote(sp, timer)
            rk.back(sp, timer)

        def all_gather():
            with torch.cuda.stream(st):
                for rk in self.ranks:
                    k = rk.batches % 2
                    for q, src in enumerate(self.ranks):
                        rk.pose_recv[k][q].copy_(src.pose_send[k])
        _timed(timer, "pose_gather", all_gather)
        for rk in self.ranks:
            rk.finish(sp, timer)

    def _step_rgbd(self, parts, st) -> None:
        torch, sp = self.torch, st.cuda_stream
        for r, rk in enumerate(self.ranks):
            rk.begin(parts[r])
            rk.front(sp)
            rk.back(sp)
            rk.pack_pairs(sp)
        with torch.cuda.stream(st):   # the all-to-all of pair blocks
            for r, rk in enumerate(self.ranks):
                k = rk.batches % 2
                for q, src in enumerate(self.ranks):
                    if q != r:
                        rk.feat_recv[k][q].copy_(src.feat_send[k][r])
        for rk in self.ranks:
            rk.rig_range(sp)
        with torch.cuda.stream(st):
            for rk in self.ranks:
                k = rk.batches % 2
                for q, src in enumerate(self.ranks):
                    rk.pose_recv[k][q].copy_(src.pose_send[k])
        for rk in self.ranks:
            rk.finish(sp)

    def read(self, rank: int = 0, n: int | None = None) -> dict:
        return self.ranks[rank].read(n)

    def close(self) -> None:
        for rk in self.ranks:
            rk.close()


class DistShardedRig:
    """One rank of a sharded rig under ``torch.distributed`` (one process per GPU).

    Backend ``nccl`` (RCCL): device buffers, asynchronous collectives ordered by stream waits —
    the raw-image all-to-all of a batch starts at once and overlaps that batch's front end, the
    front end of batch s+1 overlaps the back end of batch s (two streams), nothing blocks the
    host.  Backend ``gloo``: the same phases with host-staged, blocking collectives (CPU tests
    and a one-GPU, many-process rehearsal)."""

    def __init__(self, rects: list, cfg, batch: int, base_T_rect: list | None = None, device: int = 0,
                 exchange: str = "alltoall", front_priority: bool = True):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.plan = ShardPlan((1 if cfg.rgbd else 2) * len(rects), self.world, batch)
        self.rgbd = bool(cfg.rgbd)
        if self.rgbd:
            exchange = "alltoall"   # pair blocks go only to the rank that solves their frames
        self.rk = RankShard(rects, cfg, self.plan, self.rank, base_T_rect, device, exchange)
        self.exchange = exchange
        self.on_device = dist.get_backend() == "nccl"
        # The pose all-gather runs on a communicator of its own: one process group's collectives
        # execute in issue order on one internal stream, so a gather waiting for batch s's back
        # end would otherwise hold up batch s+1's image and stream-block exchanges behind it (the
        # exchanges then could not overlap the back end).  Every rank issues both groups'
        # collectives in the same order; RCCL kernels are a few blocks each, so the two can run
        # side by side.
        self.pose_group = dist.new_group(ranks=list(range(self.world)), backend="nccl") if self.on_device else None
        self.front_stream = torch.cuda.Stream(device=device, priority=-1 if front_priority else 0)
        self.back_stream = torch.cuda.Stream(device=device)
        self.x_stream = torch.cuda.Stream(device=device)
        self.consumed = [torch.cuda.Event(), torch.cuda.Event()]   # recv buffers of a parity read
        self.consumed_armed = [False, False]
        self.work = {"raw": [None, None], "feat": [None, None], "pose": [None, None]}

    def _collective(self, kind: str, recv, send, k: int, stream) -> None:
        torch, dist = self.torch, self.dist
        if self.on_device:
            with torch.cuda.stream(stream):
                if kind == "pose":
                    w = dist.all_gather_into_tensor(recv, send, group=self.pose_group, async_op=True)
                elif self.exchange == "allgather":
                    w = dist.all_gather_into_tensor(recv, send, async_op=True)
                else:
                    w = dist.all_to_all_single(recv, send, async_op=True)
            self.work[kind][k] = w
            return
        stream.synchronize()   # gloo: stage through the host, blocking
        hs, hr = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
        if kind == "pose" or self.exchange == "allgather":
            dist.all_gather_into_tensor(hr, hs)
        else:
            dist.all_to_all_single(hr, hs)
        recv.copy_(hr.to(recv.device))
        torch.cuda.synchronize()
        self.work[kind][k] = None

    def _wait(self, kind: str, k: int, stream) -> None:
        w = self.work[kind][k]
        if w is not None:
            with self.torch.cuda.stream(stream):
                w.wait()
            self.work[kind][k] = None

    def step(self, images, timer: StageTimer | None = None) -> None:
        """images: device u8 [B][S][H][W] of this rank's cameras (RGB-D: [B][S][5HW]), resident."""
        if self.rgbd:
            self._step_rgbd(images, timer)
            return
        rk, k = self.rk, self.rk.batches % 2
        fs, bs, xs = self.front_stream, self.back_stream, self.x_stream
        rk.begin(images)
        # the exchange buffers of this parity (raw/feature send + receive) are free once batch
        # s-2's imports ran: those waited for its collectives
        if self.consumed_armed[k]:
            xs.wait_event(self.consumed[k])
            fs.wait_event(self.consumed[k])
        # raw images: staged + sent at once (overlaps the front end)
        xs.wait_stream(self.torch.cuda.current_stream())   # the caller's input is ready
        rk.stage_raw(xs)
        self._collective("raw", rk.raw_recv[k], rk.raw_send[k], k, xs)
        # front end of this rank's cameras (high-priority stream), then its stream blocks
        if timer is not None:
            timer.stream = fs
        rk.front(fs.cuda_stream, timer)
        rk.pack_features(fs.cuda_stream)
        e_front = timer.event(fs) if timer is not None else None
        xs.wait_stream(fs)
        self._collective("feat", rk.feat_recv[k], rk.feat_send[k], k, xs)
        # back end of this rank's frame range, on the back stream, once both exchanges landed
        self._wait("raw", k, bs)
        self._wait("feat", k, bs)
        if timer is not None:
            # the exchange left exposed: front end done -> both exchanges landed on the back stream
            timer.span("exchange_exposed", e_front, timer.event(bs))
            timer.stream = bs
        rk.import_remote(bs.cuda_stream, timer)
        self.consumed[k].record(bs)
        self.consumed_armed[k] = True
        rk.back(bs.cuda_stream, timer)
        e_p = timer.event(bs) if timer is not None else None
        self._collective("pose", rk.pose_recv[k].view(-1), rk.pose_send[k].view(-1), k, bs)
        self._wait("pose", k, bs)
        if timer is not None:
            timer.span("pose_gather", e_p, timer.event(bs))
        rk.finish(bs.cuda_stream, timer)

    def _step_rgbd(self, images, timer) -> None:
        """RGB-D: own cameras' front end (front stream) and back end (back stream) over the whole
        batch, then on the back stream the pair-block all-to-all, the range's rig pose, the pose
        all-gather and the chain (the next batch's front end overlaps them)."""
        rk, k = self.rk, self.rk.batches % 2
        fs, bs = self.front_stream, self.back_stream
        rk.begin(images)
        fs.wait_stream(self.torch.cuda.current_stream())   # the caller's input is ready
        bs.wait_stream(self.torch.cuda.current_stream())   # (the depth lookup reads it too)
        if timer is not None:
            timer.stream = fs
        rk.front(fs.cuda_stream, timer)
        if timer is not None:
            timer.stream = bs
        rk.back(bs.cuda_stream, timer)
        rk.pack_pairs(bs.cuda_stream)
        e_x = timer.event(bs) if timer is not None else None
        self._collective("feat", rk.feat_recv[k], rk.feat_send[k], k, bs)
        self._wait("feat", k, bs)
        if timer is not None:
            timer.span("exchange_exposed", e_x, timer.event(bs))
        rk.rig_range(bs.cuda_stream, timer)
        e_p = timer.event(bs) if timer is not None else None
        self._collective("pose", rk.pose_recv[k].view(-1), rk.pose_send[k].view(-1), k, bs)
        self._wait("pose", k, bs)
        if timer is not None:
            timer.span("pose_gather", e_p, timer.event(bs))
        rk.finish(bs.cuda_stream, timer)

    def drain(self) -> None:
        for kind in self.work:
            for k in (0, 1):
                self._wait(kind, k, self.back_stream)
        self.torch.cuda.synchronize()

    def read(self, n: int | None = None) -> dict:
        self.drain()
        return self.rk.read(n)

    def close(self) -> None:
        self.rk.close()
