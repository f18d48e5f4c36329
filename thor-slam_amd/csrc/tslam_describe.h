// tslam_describe.h — tile geometry of k_describe, shared with the host (BRIEF offset table).
#pragma once

#define TS_DT_W 128                         // tile columns
#define TS_DT_H 32                          // tile rows
#define TS_DT_HX 32                         // column halo: >= 18 and keeps 16-byte alignment
// LDS pitch (and staged width) of both images: 208 = 13 x 16 B.  The 16 extra columns move the
// rows against the 64 LDS banks: the rotated BRIEF reads of a wave conflict ~2.5-way instead of
// ~4.6-way at pitch 192 (all 30 bins, both points; tools/brief_banks.py)
#ifndef TS_DT_PAD
#define TS_DT_PAD 16
#endif
#define TS_DT_P (TS_DT_W + 2 * TS_DT_HX + TS_DT_PAD)
#define TS_DT_RAW_ROWS (TS_DT_H + 30)       // raw level: orientation disc radius 15
#define TS_DT_SMO_ROWS (TS_DT_H + 36)       // smoothed level: rotated BRIEF radius 18
