// tslam_describe.h — tile geometry of k_describe, shared with the host (BRIEF offset table).
#pragma once

#define TS_DT_W 128                         // tile columns
// 128 x 64 tiles on 8 waves: the row halos are staged for 64 rows instead of 32 and the LDS
// (44 KB) still holds 3 blocks = 6 waves per SIMD (461 -> 446 us per 256-frame batch alone;
// 128 x 32 on 8 waves 517, 128 x 64 on 4 waves 501)
#ifndef TS_DT_H
#define TS_DT_H 64                          // tile rows
#endif
#ifndef TS_DT_THREADS
#define TS_DT_THREADS 512                   // threads per describe block
#endif
#define TS_DT_HX 32                         // column halo: >= 18 and keeps 16-byte alignment
// LDS pitch (and staged width) of both images: 208 = 13 x 16 B.  The 16 extra columns move the
// rows against the 64 LDS banks: the rotated BRIEF reads of a wave conflict ~2.5-way instead of
// ~4.6-way at pitch 192 (all 30 bins, both points; tools/brief_banks.py)
#ifndef TS_DT_PAD
#define TS_DT_PAD 16
#endif
#define TS_DT_P (TS_DT_W + 2 * TS_DT_HX + TS_DT_PAD)
#define TS_DT_RAW_ROWS (TS_DT_H + 30)       // raw level: orientation disc radius 15
#define TS_DT_RAW_P 160                     // raw tile pitch: columns [x0 - 16, x0 + 144), 10 x 16 B
#define TS_DT_SMO_ROWS (TS_DT_H + 36)       // smoothed level: rotated BRIEF radius 18
