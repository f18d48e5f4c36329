// host_check.cpp — the library's host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer
// (`make -C thor-slam_amd/csrc sanitize`; tests/test_sanitizers.py).  Linked with the host sources
// themselves (tslam_calib.cpp, tslam_imu.cpp, tslam_ranges.h) — not with libtslam_hip.so — so the
// sanitizer runtime comes first in this executable and nothing has to be preloaded.
//
//   host_check maps  calib.txt out.bin   tslam_rig_pairs + tslam_rectify_pair (rig_from_calib.c's format)
//   host_check imu   script.bin out.bin  the tslam_imu_* filter over a scripted sequence
//   host_check ranges                    the sharded frame-range arithmetic, exhaustively
// Exit status 0 on success; a sanitizer report aborts (-fno-sanitize-recover=all).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tslam.h"
#include "../../thor-slam_amd/csrc/tslam_ranges.h"

// tslam_api.cpp's error setter (the host sources report through it)
static std::string g_err;
int tslam_internal_fail(int code, const char* msg) {
    g_err = msg;
    return code;
}
// tslam_create_rig (tslam_calib.cpp) creates a device handle: not part of the host check; its
// section is dropped by --gc-sections, these keep a non-gc link (e.g. -O0 builds) resolvable
extern "C" int tslam_create(const tslam_stereo_desc*, const tslam_params*, int, tslam_handle**) { return TSLAM_ESTATE; }
extern "C" int tslam_set_rig(tslam_handle*, const double*) { return TSLAM_ESTATE; }
extern "C" int tslam_destroy(tslam_handle*) { return TSLAM_OK; }

static int die(const char* what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, g_err.c_str());
    return 1;
}

static std::vector<uint8_t> slurp(const char* path) {
    std::vector<uint8_t> v;
    FILE* f = fopen(path, "rb");
    if (!f) return v;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    fclose(f);
    return v;
}

// calib.txt: one camera per line (tests/native_caller.py write_calib)
static int read_calib(const char* path, std::vector<tslam_camera_desc>& cams, std::vector<std::string>& names) {
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    char name[256];
    tslam_camera_desc c{};
    while (fscanf(f, "%255s %d %d %d %d", name, &c.cam_idx, &c.width, &c.height, &c.n_coeffs) == 5) {
        for (double& v : c.K)
            if (fscanf(f, "%lf", &v) != 1) return -1;
        for (double& v : c.D)
            if (fscanf(f, "%lf", &v) != 1) return -1;
        for (double& v : c.world_T_cam)
            if (fscanf(f, "%lf", &v) != 1) return -1;
        names.emplace_back(name);
        cams.push_back(c);
    }
    fclose(f);
    for (size_t i = 0; i < cams.size(); ++i) cams[i].source = names[i].c_str();
    return (int)cams.size();
}

static int cmd_maps(const char* calib, const char* out_path) {
    std::vector<tslam_camera_desc> cams;
    std::vector<std::string> names;
    names.reserve(64);
    if (read_calib(calib, cams, names) < 1) return die("read calib", -1);
    std::vector<int32_t> pairs(2 * cams.size());
    const int np = tslam_rig_pairs(cams.data(), (int)cams.size(), pairs.data(), (int)cams.size());
    if (np < 0) return die("tslam_rig_pairs", np);
    FILE* out = fopen(out_path, "wb");
    if (!out) return die("open out", -1);
    for (int p = 0; p < np; ++p) {
        const tslam_camera_desc& L = cams[pairs[2 * p]];
        const tslam_camera_desc& R = cams[pairs[2 * p + 1]];
        const size_t cells = (size_t)L.width * L.height * 2;
        std::vector<int32_t> ml(cells), mr(cells);
        tslam_stereo_desc d{};
        double base[16];
        const int rc = tslam_rectify_pair(&L, &R, &d, ml.data(), mr.data(), base, nullptr);
        if (rc) return die("tslam_rectify_pair", rc);
        const double sc[5] = {d.fx, d.fy, d.cx, d.cy, d.baseline};
        fwrite(&pairs[2 * p], 4, 2, out);
        fwrite(sc, 8, 5, out);
        fwrite(base, 8, 16, out);
        fwrite(ml.data(), 4, cells, out);
        fwrite(mr.data(), 4, cells, out);
    }
    fclose(out);
    return 0;
}

// script.bin: i32 accel, i32 n_batches, f64 rect_R_imu[9], noise[TSLAM_IMU_NOISE], lever[3],
// begin_accel[3]; per batch: i32 n, i32 0, f64 dt[n], gyro[n][3], accel[n][3], t_rel[n][16],
// cov[n][36], i32 status[n] (padded to 8 bytes).  out.bin: per batch the priors (tslam_imu_step[n], i32 valid[n])
// and the state after tslam_imu_absorb (tslam_imu_state).
struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;
    template <class T>
    const T* take(size_t n) {
        const size_t b = n * sizeof(T);
        if ((size_t)(end - p) < b) {
            ok = false;
            return nullptr;
        }
        const T* r = reinterpret_cast<const T*>(p);
        p += b;
        return r;
    }
};

static int cmd_imu(const char* script, const char* out_path) {
    const std::vector<uint8_t> raw = slurp(script);
    Reader rd{raw.data(), raw.data() + raw.size()};
    const int32_t* hdr = rd.take<int32_t>(2);
    const double* ri = rd.take<double>(9);
    const double* noise = rd.take<double>(TSLAM_IMU_NOISE);
    const double* lever = rd.take<double>(3);
    const double* a0 = rd.take<double>(3);
    if (!rd.ok) return die("read script header", -1);
    tslam_imu* f = nullptr;
    int rc = tslam_imu_create(ri, noise, lever, hdr[0], &f);
    if (rc) return die("tslam_imu_create", rc);
    const bool accel = hdr[0] != 0;   // the gyro-only filter takes no accelerometer samples
    if ((rc = tslam_imu_begin(f, accel ? a0 : nullptr))) return die("tslam_imu_begin", rc);
    FILE* out = fopen(out_path, "wb");
    if (!out) return die("open out", -1);
    for (int b = 0; b < hdr[1]; ++b) {
        const int32_t n = *rd.take<int32_t>(2);   // n, pad: the doubles stay 8-byte aligned
        const double* dt = rd.take<double>(n);
        const double* gy = rd.take<double>(3 * (size_t)n);
        const double* ac = rd.take<double>(3 * (size_t)n);
        const double* tr = rd.take<double>(16 * (size_t)n);
        const double* cv = rd.take<double>(36 * (size_t)n);
        const int32_t* st = rd.take<int32_t>(n + (n & 1));   // padded to 8 bytes
        if (!rd.ok) return die("read script batch", -1);
        std::vector<tslam_imu_step> steps(n);
        std::vector<int32_t> valid(n);
        if ((rc = tslam_imu_batch_priors(f, n, dt, gy, accel ? ac : nullptr, steps.data(), valid.data())))
            return die("batch_priors", rc);
        if ((rc = tslam_imu_absorb(f, n, dt, gy, accel ? ac : nullptr, st, tr, cv))) return die("absorb", rc);
        tslam_imu_state s{};
        if ((rc = tslam_imu_get_state(f, &s))) return die("get_state", rc);
        fwrite(steps.data(), sizeof(tslam_imu_step), n, out);
        fwrite(valid.data(), 4, n, out);
        fwrite(&s, sizeof s, 1, out);
    }
    fclose(out);
    tslam_imu_destroy(f);
    return 0;
}

// Every (n, world) with 1 <= world <= max_batch <= 1024: the ranges partition the batch in order,
// differ in length by at most one, fit the per-peer slot and the padded all-gather.
static int cmd_ranges() {
    long checked = 0;
    for (int B = 1; B <= 1024; B = B < 64 ? B + 1 : B * 2) {
        for (int world = 1; world <= std::min(B, 64); ++world) {
            const int cap = peer_cap(B, world);
            for (int n = 1; n <= B; ++n) {
                int prev_hi = 0, mn = 1 << 30, mx = -1;
                const int recs = peer_records(n, world);
                for (int q = 0; q < world; ++q) {
                    int lo, hi;
                    peer_range(q, n, world, &lo, &hi);
                    if (lo != prev_hi || hi < lo || hi > n) return die("ranges: not a partition", q);
                    prev_hi = hi;
                    mn = std::min(mn, hi - lo);
                    mx = std::max(mx, hi - lo);
                    const int fr = peer_frames(q, n, world);
                    if (fr > cap || (hi > lo ? fr != hi - lo + 1 : fr != 0)) return die("ranges: frames vs slot", q);
                    if (hi - lo > recs) return die("ranges: records", q);
                    ++checked;
                }
                if (prev_hi != n || mx - mn > 1) return die("ranges: uneven", n);
                // pair split (even world = cameras): rig_rank inverts rig_slot, and every rank's rig
                // range lies inside its pair's half, which fits the stereo receive buffers
                if (world % 2 || world < 2) continue;
                for (int r = 0; r < world; ++r) {
                    const int sl = rig_slot(r, world, 1);
                    if (sl < 0 || sl >= world || rig_rank(sl, world, 1) != r) return die("pairs: slot", r);
                    int lo, hi, hlo, hhi;
                    peer_range(sl, n, world, &lo, &hi);
                    peer_range(r & 1, n, 2, &hlo, &hhi);
                    if (hi > lo && (lo < hlo || hi > hhi)) return die("pairs: rig range outside the half", r);
                    if ((hhi > hlo ? hhi - hlo + 1 : 0) > world * cap) return die("pairs: half vs receive slots", r);
                    ++checked;
                }
            }
        }
    }
    printf("ranges: %ld (rank, n, world, max_batch) cases\n", checked);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 4 && !strcmp(argv[1], "maps")) return cmd_maps(argv[2], argv[3]);
    if (argc >= 4 && !strcmp(argv[1], "imu")) return cmd_imu(argv[2], argv[3]);
    if (argc >= 2 && !strcmp(argv[1], "ranges")) return cmd_ranges();
    fprintf(stderr, "usage: host_check maps calib.txt out.bin | imu script.bin out.bin | ranges\n");
    return 2;
}
