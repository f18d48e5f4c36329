// tslam_internal.h — what the library's host files share beyond the public C-ABI (include/tslam.h):
// the error setter, a read-only view of a handle's geometry, and the attachment of a sharded-rig
// driver (tslam_shard.cpp) to the handles it drives.
#pragma once

#include <stdint.h>

#include "../../include/tslam.h"

struct tslam_shard_driver;   // tslam_shard.cpp

#define TSLAM_INTERNAL __attribute__((visibility("hidden")))

// sets tslam_last_error() and returns `code`
int tslam_internal_fail(int code, const char* msg);

// not exported from libtslam_hip.so (only include/tslam.h is its ABI)
extern "C" {
struct tslam_handle_info {
    int device, W, H, P, C, B, rgbd, rig, ba;
    int64_t frames_done;
    int64_t stream_block, pose_record, pair_block;   // exchange unit sizes (bytes)
    int cam_lo, cam_hi, rank, world;                 // tslam_set_shard
};
TSLAM_INTERNAL int tslam_internal_info(tslam_handle* h, tslam_handle_info* out);

// `owned`: the handle destroys the driver with itself (tslam_comm_init); a group's driver is owned
// by the group (tslam_group_destroy detaches it first).  NULL detaches.
TSLAM_INTERNAL int tslam_internal_attach_driver(tslam_handle* h, tslam_shard_driver* d, bool owned);
TSLAM_INTERNAL tslam_shard_driver* tslam_internal_driver(tslam_handle* h);
TSLAM_INTERNAL void tslam_internal_driver_destroy(tslam_shard_driver* d);

// State gather of a sharded stereo rig (k_exchange.hip, state blocks): bytes of sender `rank`'s
// payload for an n-frame batch; pack (on the sender, its own rank / cameras) or unpack (on rank 0,
// the sender's rank and camera range) inside a batch, after the back end of the sender's range.
TSLAM_INTERNAL int64_t tslam_internal_state_bytes(tslam_handle* h, int n, int rank, int cam_lo, int cam_hi);
TSLAM_INTERNAL int tslam_internal_state_blocks(tslam_handle* h, int pack, int rank, int cam_lo, int cam_hi, void* buf,
                                               void* stream);
// the current batch's poses / stats into the handle's pinned result slots (tslam_poll_batch)
TSLAM_INTERNAL int tslam_internal_stash(tslam_handle* h, void* stream);

// Pair split (TSLAM_SHARD_PAIRS, tslam_ranges.h rig_slot): set / clear it on a sharded stereo
// handle with one camera per rank (outside a batch).  Inside a batch: pack this camera's stream
// blocks of the partner's half (frames lo' - 1 .. hi' - 1, the partner = the pair's other camera)
// -> dst; import the partner's raw images + stream blocks of this rank's half (as received) into
// the ring.  Pair blocks of the rig ranges move with tslam_pack_pairs / tslam_unpack_pairs.
TSLAM_INTERNAL int tslam_internal_set_pairs(tslam_handle* h, int on);
TSLAM_INTERNAL int tslam_internal_pack_partner(tslam_handle* h, void* dst, void* stream);
TSLAM_INTERNAL int tslam_internal_import_partner(tslam_handle* h, const uint8_t* raw, const void* streams, void* stream);
}  // extern "C"
