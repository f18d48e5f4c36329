// tslam_describe.h — tile geometry of k_describe, shared with the host (BRIEF offset table).
#pragma once

#define TS_DT_W 128                         // tile columns
#define TS_DT_H 32                          // tile rows
#define TS_DT_HX 32                         // column halo: >= 18 and keeps 16-byte alignment
#define TS_DT_P (TS_DT_W + 2 * TS_DT_HX)    // LDS pitch of both staged images (192)
#define TS_DT_RAW_ROWS (TS_DT_H + 30)       // raw level: orientation disc radius 15
#define TS_DT_SMO_ROWS (TS_DT_H + 36)       // smoothed level: rotated BRIEF radius 18
