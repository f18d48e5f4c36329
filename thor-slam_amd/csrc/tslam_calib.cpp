// Host-side calibration behind tslam_create_rig: rows A1/A2 of SURVEY.md §8a in C++, so a native
// caller hands the library the raw camera_info of every camera (K, D, world extrinsics) the way
// IsaacRosAdapter publishes it (thor_slam/slam/adapters/isaac_ros.py:364-411) and gets the same
// handle HipSlamEngine.initialize builds through thor_slam_amd/calib.py.
//
// Every function restates one of calib.py (the spec; the test compares the two byte for byte):
//   camera order + pairing    extract_cameras / stereo_pairs   (isaac_ros.py:138-157)
//   distortion model          distortion_model                 (isaac_ros.py:370-383)
//   distortion                distort_normalized
//   remap table               rectify_map   (1/32-px fixed point, RECT_FRAC_BITS = 5)
//   Bouguet rectification     stereo_rectify
//   RGB-D undistortion        rgbd_undistort
// Rotations follow the quaternion algorithms scipy.spatial.transform.Rotation uses (from_matrix,
// as_rotvec, from_rotvec, as_matrix), so the rectifying rotations agree to the last bits.
// Built with -ffp-contract=off like the rest of the library: no fused multiply-adds, the
// operation order of each numpy expression is kept.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/tslam.h"

int tslam_internal_fail(int code, const char* msg);   // tslam_api.cpp: sets tslam_last_error()

namespace {

constexpr int RECT_FRAC_BITS = 5;
constexpr int RECT_ONE = 1 << RECT_FRAC_BITS;

struct Mat3 {
    double m[3][3];
};

Mat3 mul(const Mat3& a, const Mat3& b) {
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return r;
}

Mat3 transpose(const Mat3& a) {
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
    return r;
}

void mulv(const Mat3& a, const double v[3], double out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = a.m[i][0] * v[0] + a.m[i][1] * v[1] + a.m[i][2] * v[2];
}

double norm3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// scipy Rotation.from_rotvec(v).as_matrix()
Mat3 rot_from_rotvec(const double v[3]) {
    const double angle = norm3(v);
    double scale;
    if (angle <= 1e-3) {
        const double a2 = angle * angle;
        scale = 0.5 - a2 / 48.0 + a2 * a2 / 3840.0;
    } else {
        scale = std::sin(angle / 2.0) / angle;
    }
    const double x = scale * v[0], y = scale * v[1], z = scale * v[2], w = std::cos(angle / 2.0);
    const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
    const double xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
    Mat3 r;
    r.m[0][0] = x2 - y2 - z2 + w2;
    r.m[1][0] = 2 * (xy + zw);
    r.m[2][0] = 2 * (xz - yw);
    r.m[0][1] = 2 * (xy - zw);
    r.m[1][1] = -x2 + y2 - z2 + w2;
    r.m[2][1] = 2 * (yz + xw);
    r.m[0][2] = 2 * (xz + yw);
    r.m[1][2] = 2 * (yz - xw);
    r.m[2][2] = -x2 - y2 + z2 + w2;
    return r;
}

// scipy Rotation.from_matrix(m).as_rotvec(): quaternion from the largest of (diag, trace), then
// the canonical (w >= 0) axis-angle
void rotvec_from_rot(const Mat3& a, double out[3]) {
    const double* m[3] = {a.m[0], a.m[1], a.m[2]};
    const double dec[4] = {m[0][0], m[1][1], m[2][2], m[0][0] + m[1][1] + m[2][2]};
    int choice = 0;
    for (int i = 1; i < 4; ++i)
        if (dec[i] > dec[choice]) choice = i;
    double q[4];
    if (choice != 3) {
        const int i = choice, j = (i + 1) % 3, k = (j + 1) % 3;
        q[i] = 1 - dec[3] + 2 * m[i][i];
        q[j] = m[j][i] + m[i][j];
        q[k] = m[k][i] + m[i][k];
        q[3] = m[k][j] - m[j][k];
    } else {
        q[0] = m[2][1] - m[1][2];
        q[1] = m[0][2] - m[2][0];
        q[2] = m[1][0] - m[0][1];
        q[3] = 1 + dec[3];
    }
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double& c : q) c /= n;
    if (q[3] < 0)
        for (double& c : q) c = -c;
    const double v[3] = {q[0], q[1], q[2]};
    const double angle = 2 * std::atan2(norm3(v), q[3]);
    double scale;
    if (angle <= 1e-3) {
        const double a2 = angle * angle;
        scale = 2 + a2 / 12 + 7 * a2 * a2 / 2880;
    } else {
        scale = angle / std::sin(angle / 2);
    }
    for (int i = 0; i < 3; ++i) out[i] = scale * q[i];
}

// calib.distortion_model (isaac_ros.py:370-383): >= 8 coefficients -> rational_polynomial[:8],
// 5 -> plumb_bob, 4 -> equidistant, otherwise plumb_bob zero-padded / cut to 5
struct Distortion {
    bool equidistant;
    double k[8];
};

Distortion distortion_model(const double* d, int n) {
    Distortion r{};
    if (n >= 8) {
        std::copy(d, d + 8, r.k);
    } else if (n == 4) {
        r.equidistant = true;
        std::copy(d, d + 4, r.k);
    } else {
        std::copy(d, d + std::min(n, 5), r.k);
    }
    return r;
}

// calib.distort_normalized, numpy's evaluation order
void distort(const Distortion& dm, double x, double y, double* xd, double* yd) {
    if (dm.equidistant) {
        const double k1 = dm.k[0], k2 = dm.k[1], k3 = dm.k[2], k4 = dm.k[3];
        const double r = std::sqrt(x * x + y * y);
        const double th = std::atan(r);
        const double th2 = th * th;
        const double thd = th * (1 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4))));
        const double scale = r > 1e-12 ? thd / r : 1.0;
        *xd = x * scale;
        *yd = y * scale;
        return;
    }
    const double k1 = dm.k[0], k2 = dm.k[1], p1 = dm.k[2], p2 = dm.k[3], k3 = dm.k[4], k4 = dm.k[5], k5 = dm.k[6],
                 k6 = dm.k[7];
    const double r2 = x * x + y * y;
    const double radial = (1 + r2 * (k1 + r2 * (k2 + r2 * k3))) / (1 + r2 * (k4 + r2 * (k5 + r2 * k6)));
    *xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x);
    *yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y;
}

int32_t fixed(double s, double lim) {
    double v = std::floor(s * RECT_ONE + 0.5);
    v = std::min(std::max(v, -2.0 * RECT_ONE), lim);
    return (int32_t)v;
}

// calib.rectify_map: rectified pixel -> raw pixel of this camera, (x, y) * 32, [H][W][2]
void rectify_map(const tslam_camera_desc& cam, const Mat3& rect_rot, double fx, double fy, double cx, double cy,
                 int32_t* map) {
    const int w = cam.width, h = cam.height;
    const Distortion dm = distortion_model(cam.D, cam.n_coeffs);
    const double* k = cam.K;
    const double lim_x = (double)(w + 1) * RECT_ONE, lim_y = (double)(h + 1) * RECT_ONE;
    for (int v = 0; v < h; ++v) {
        for (int u = 0; u < w; ++u) {
            const double a0 = ((double)u - cx) / fx, a1 = ((double)v - cy) / fy;
            double ray[3];   // row vector @ rect_rot (R^T applied)
            for (int j = 0; j < 3; ++j) ray[j] = a0 * rect_rot.m[0][j] + a1 * rect_rot.m[1][j] + rect_rot.m[2][j];
            const double xn = ray[0] / ray[2], yn = ray[1] / ray[2];
            double xd, yd;
            distort(dm, xn, yn, &xd, &yd);
            const double su = k[0] * xd + k[1] * yd + k[2];
            const double sv = k[4] * yd + k[5];
            int32_t* o = map + ((size_t)v * w + u) * 2;
            o[0] = fixed(su, lim_x);
            o[1] = fixed(sv, lim_y);
        }
    }
}

bool is_identity_map(const int32_t* map, int w, int h) {
    for (int v = 0; v < h; ++v)
        for (int u = 0; u < w; ++u) {
            const int32_t* o = map + ((size_t)v * w + u) * 2;
            if (o[0] != u * RECT_ONE || o[1] != v * RECT_ONE) return false;
        }
    return true;
}

Mat3 rot_of(const double* T) {
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = T[4 * i + j];
    return r;
}

bool valid_camera(const tslam_camera_desc* c) {
    return c && c->width > 0 && c->height > 0 && c->n_coeffs >= 0 && c->n_coeffs <= 14;
}

// world_T_cam(left) @ [rect^T | 0]: the rectified-left frame in the rig's base frame
void base_T_rect_of(const tslam_camera_desc& left, const Mat3& rect_left, double* out) {
    const Mat3 rt = transpose(rect_left);
    const double* T = left.world_T_cam;
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 3; ++j) out[4 * i + j] = T[4 * i + 0] * rt.m[0][j] + T[4 * i + 1] * rt.m[1][j] + T[4 * i + 2] * rt.m[2][j];
        out[4 * i + 3] = T[4 * i + 3];
    }
}

}  // namespace

extern "C" int tslam_rectify_pair(const tslam_camera_desc* left, const tslam_camera_desc* right, tslam_stereo_desc* desc,
                                  int32_t* map_left, int32_t* map_right, double* base_T_rect, double* rect_rot) {
    if (!valid_camera(left) || !valid_camera(right) || !desc)
        return tslam_internal_fail(TSLAM_EINVAL, "tslam_rectify_pair: bad camera description");
    if (left->width != right->width || left->height != right->height)
        return tslam_internal_fail(TSLAM_EINVAL, "stereo pair cameras must share the image size");
    // relative pose r_T_l from the two world extrinsics (rigid inverse, calib.stereo_rectify)
    const Mat3 rl = rot_of(left->world_T_cam), rr = rot_of(right->world_T_cam);
    const double tl[3] = {left->world_T_cam[3], left->world_T_cam[7], left->world_T_cam[11]};
    const double tr[3] = {right->world_T_cam[3], right->world_T_cam[7], right->world_T_cam[11]};
    const Mat3 rlt = transpose(rl);
    const Mat3 l_R_r = mul(rlt, rr);
    const double dt[3] = {tr[0] - tl[0], tr[1] - tl[1], tr[2] - tl[2]};
    double l_t_r[3];
    mulv(rlt, dt, l_t_r);
    const Mat3 rot = transpose(l_R_r);   // r_R_l
    double trans[3];
    mulv(rot, l_t_r, trans);
    for (double& c : trans) c = -c;      // r_t_l = -r_R_l l_t_r

    double om[3];
    rotvec_from_rot(rot, om);
    const double half[3] = {-0.5 * om[0], -0.5 * om[1], -0.5 * om[2]};
    const Mat3 r_r = rot_from_rotvec(half);
    double t[3];
    mulv(r_r, trans, t);
    const int idx = std::fabs(t[0]) > std::fabs(t[1]) ? 0 : 1;
    double uu[3] = {0, 0, 0};
    uu[idx] = t[idx] > 0 ? 1.0 : -1.0;
    double ww[3] = {t[1] * uu[2] - t[2] * uu[1], t[2] * uu[0] - t[0] * uu[2], t[0] * uu[1] - t[1] * uu[0]};
    const double nw = norm3(ww);
    if (nw > 0.0) {
        const double s = std::acos(std::min(1.0, std::fabs(t[idx]) / norm3(t))) / nw;
        for (double& c : ww) c = c * s;
    }
    const Mat3 w_r = rot_from_rotvec(ww);
    const Mat3 rect_l = mul(w_r, transpose(r_r));
    const Mat3 rect_r = mul(w_r, r_r);
    double t_new[3];
    mulv(rect_r, trans, t_new);

    const double* kl = left->K;
    const double* kr = right->K;
    const double f = std::min(std::min(kl[0], kl[4]), std::min(kr[0], kr[4]));
    const double cx = 0.5 * (kl[2] + kr[2]), cy = 0.5 * (kl[5] + kr[5]);
    desc->width = left->width;
    desc->height = left->height;
    desc->fx = desc->fy = f;
    desc->cx = cx;
    desc->cy = cy;
    desc->baseline = -t_new[0];
    desc->map_left = map_left;
    desc->map_right = map_right;
    if (map_left) rectify_map(*left, rect_l, f, f, cx, cy, map_left);
    if (map_right) rectify_map(*right, rect_r, f, f, cx, cy, map_right);
    if (base_T_rect) base_T_rect_of(*left, rect_l, base_T_rect);
    if (rect_rot) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                rect_rot[3 * i + j] = rect_l.m[i][j];
                rect_rot[9 + 3 * i + j] = rect_r.m[i][j];
            }
    }
    return TSLAM_OK;
}

extern "C" int tslam_rgbd_undistort(const tslam_camera_desc* color, tslam_stereo_desc* desc, int32_t* map,
                                    double* base_T_rect) {
    if (!valid_camera(color) || !desc) return tslam_internal_fail(TSLAM_EINVAL, "tslam_rgbd_undistort: bad camera description");
    const double* k = color->K;
    const double f = std::min(k[0], k[4]);
    Mat3 eye{};
    for (int i = 0; i < 3; ++i) eye.m[i][i] = 1.0;
    desc->width = color->width;
    desc->height = color->height;
    desc->fx = desc->fy = f;
    desc->cx = k[2];
    desc->cy = k[5];
    desc->baseline = 1.0;
    desc->map_left = desc->map_right = map;
    if (map) rectify_map(*color, eye, f, f, k[2], k[5], map);
    if (base_T_rect) base_T_rect_of(*color, eye, base_T_rect);
    return TSLAM_OK;
}

extern "C" int tslam_rig_pairs(const tslam_camera_desc* cams, int n_cams, int32_t* pairs, int max_pairs) {
    if (!cams || n_cams < 0) return tslam_internal_fail(TSLAM_EINVAL, "tslam_rig_pairs: bad camera list");
    // extract_cameras: sources in sorted name order, each source's cameras in the given order
    std::vector<int> order(n_cams);
    std::iota(order.begin(), order.end(), 0);
    auto name = [&](int i) { return cams[i].source ? cams[i].source : ""; };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return std::strcmp(name(a), name(b)) < 0; });
    int n = 0;
    for (int p = 1; p < n_cams; ++p) {   // stereo_pairs: cam_idx 1 directly after cam_idx 0 of its source
        const int i = order[p], prev = order[p - 1];
        if (cams[i].cam_idx == 1 && cams[prev].cam_idx == 0 && std::strcmp(name(i), name(prev)) == 0) {
            if (pairs && n < max_pairs) {
                pairs[2 * n] = prev;
                pairs[2 * n + 1] = i;
            }
            ++n;
        }
    }
    return n;
}

extern "C" int tslam_create_rig(const tslam_camera_desc* cams, int n_cams, const tslam_params* params, int device,
                                tslam_handle** out) {
    if (!params || !out) return tslam_internal_fail(TSLAM_EINVAL, "tslam_create_rig: null argument");
    for (int i = 0; i < n_cams; ++i)
        if (!valid_camera(cams + i)) return tslam_internal_fail(TSLAM_EINVAL, "tslam_create_rig: bad camera description");
    const int np = tslam_rig_pairs(cams, n_cams, nullptr, 0);
    if (np < 0) return np;
    if (np == 0)
        return tslam_internal_fail(TSLAM_EINVAL, params->rgbd ? "tslam_create_rig: no RGB-D source (colour cam_idx 0, depth cam_idx 1)"
                                                              : "tslam_create_rig: no stereo source (cam_idx 0 and 1)");
    if (params->n_pairs != 0 && params->n_pairs != np)
        return tslam_internal_fail(TSLAM_EINVAL, "tslam_create_rig: params->n_pairs disagrees with the cameras' pairs");
    std::vector<int32_t> pairs(2 * np);
    tslam_rig_pairs(cams, n_cams, pairs.data(), np);
    std::vector<tslam_stereo_desc> descs(np);
    std::vector<std::vector<int32_t>> maps;
    std::vector<double> base(16 * (size_t)np);
    for (int p = 0; p < np; ++p) {
        const tslam_camera_desc& l = cams[pairs[2 * p]];
        const tslam_camera_desc& r = cams[pairs[2 * p + 1]];
        const size_t cells = (size_t)l.width * l.height * 2;
        maps.emplace_back(cells);
        int rc;
        if (params->rgbd) {
            rc = tslam_rgbd_undistort(&l, &descs[p], maps.back().data(), &base[16 * p]);
        } else {
            maps.emplace_back(cells);
            rc = tslam_rectify_pair(&l, &r, &descs[p], maps[maps.size() - 2].data(), maps.back().data(), &base[16 * p], nullptr);
        }
        if (rc) return rc;
        // identity tables are passed as NULL (the kernel's copy path), as HipSlamEngine does
        const bool ident = is_identity_map(descs[p].map_left, l.width, l.height) &&
                           (params->rgbd || is_identity_map(descs[p].map_right, l.width, l.height));
        if (ident) descs[p].map_left = descs[p].map_right = nullptr;
    }
    tslam_params pr = *params;
    pr.n_pairs = np;
    tslam_handle* h = nullptr;
    int rc = tslam_create(descs.data(), &pr, device, &h);
    if (rc) return rc;
    if (np > 1 && (rc = tslam_set_rig(h, base.data()))) {
        tslam_destroy(h);
        return rc;
    }
    *out = h;
    return TSLAM_OK;
}
