// tslam_ranges.h — the frame-range arithmetic of a sharded rig, shared by the
// kernels (k_exchange.hip), the library's host code (tslam_api.cpp, tslam_shard.cpp) and the
// sanitizer build of the host code (tests/c/host_check.cpp, `make sanitize`): no HIP dependency.
//
// Rank q's back end owns batch frames [q n / world, (q + 1) n / world) of an n-frame batch (any n
// in [1, max_batch]: ranges may differ by one frame or be empty) and reads the other cameras of
// frames lo - 1 .. hi - 1 (none for an empty range).  Exchange slots are sized for a full batch:
// peer_cap frames per peer; the pose all-gather pads every range to peer_records records.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define TS_RANGE_HD __host__ __device__
#else
#define TS_RANGE_HD
#endif

static inline TS_RANGE_HD void peer_range(int q, int n, int world, int* lo, int* hi) {
    *lo = (int)((int64_t)q * n / world);
    *hi = (int)((int64_t)(q + 1) * n / world);
}
static inline TS_RANGE_HD int peer_frames(int q, int n, int world) {
    int lo, hi;
    peer_range(q, n, world, &lo, &hi);
    return hi > lo ? hi - lo + 1 : 0;
}
static inline TS_RANGE_HD int peer_cap(int max_batch, int world) { return (max_batch + world - 1) / world + 1; }
static inline TS_RANGE_HD int peer_records(int n, int world) { return (n + world - 1) / world; }

// Pair split (TSLAM_SHARD_PAIRS; one camera per rank, world = cameras): rank r holds camera r of
// pair r / 2 and its back end solves that pair over half of the batch, side r & 1 =
// peer_range(r & 1, n, 2).  Its rig range (rig pose + pose records) is range `rig_slot` of the
// world-way split: the even ranks take the first half's world/2 ranges in pair order, the odd
// ranks the second half's, so a rank's rig range lies inside its own half (floor ranges nest:
// peer_range(s, n, world) for s < world/2 ends by n/2) and its pair's blocks never leave it.
static inline TS_RANGE_HD int rig_slot(int rank, int world, int pairs) {
    return pairs ? (rank & 1) * (world / 2) + (rank >> 1) : rank;
}
static inline TS_RANGE_HD int rig_rank(int slot, int world, int pairs) {   // inverse of rig_slot
    return !pairs ? slot : slot < world / 2 ? 2 * slot : 2 * (slot - world / 2) + 1;
}
