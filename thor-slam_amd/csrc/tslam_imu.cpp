// tslam_imu.cpp — the IMU filter behind the motion priors, native host code.
//
// The reference fuses the OAK IMU inside cuVSLAM (enable_imu_fusion:=true, Makefile:81; samples
// in SynchronizedFrameSet.sensor_data, thor_slam/camera/types.py:268-269, rig.py:403-407; noise
// model launch/thor_visual_slam.launch.py:82-90).  This file is the product's filter: a small
// inertial state (camera orientation, world velocity, gravity, accelerometer and gyroscope biases
// and their variances) that turns each frame's sample into the prior tslam_set_motion_prior takes,
// and absorbs the tracked motions after each batch.  Spec and operation order: oracle/numpy_imu.py
// (thor_slam_amd/imu.py binds this file).  All arithmetic f64.
#include <cmath>
#include <cstring>

#include "../../include/tslam.h"

int tslam_internal_fail(int code, const char* msg);   // tslam_api.cpp: sets tslam_last_error()

namespace {

constexpr double kGravity = 9.81;

struct V3 {
    double x, y, z;
};
inline V3 v3(const double* p) { return {p[0], p[1], p[2]}; }
inline void put(const V3& a, double* p) {
    p[0] = a.x;
    p[1] = a.y;
    p[2] = a.z;
}
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double norm(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

// 3x3 row-major
inline V3 mv(const double* M, V3 a) {
    return {M[0] * a.x + M[1] * a.y + M[2] * a.z, M[3] * a.x + M[4] * a.y + M[5] * a.z,
            M[6] * a.x + M[7] * a.y + M[8] * a.z};
}
inline V3 mtv(const double* M, V3 a) {   // M^T a
    return {M[0] * a.x + M[3] * a.y + M[6] * a.z, M[1] * a.x + M[4] * a.y + M[7] * a.z,
            M[2] * a.x + M[5] * a.y + M[8] * a.z};
}
inline void mm(const double* A, const double* B, double* out) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    std::memcpy(out, t, sizeof t);
}
inline void mmt(const double* A, const double* B, double* out) {   // A B^T
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[3 * j] + A[3 * i + 1] * B[3 * j + 1] + A[3 * i + 2] * B[3 * j + 2];
    std::memcpy(out, t, sizeof t);
}

// exp of the rotation vector w (Rodrigues; series below 1e-4 rad)
void rotvec_to_matrix(V3 w, double* R) {
    const double t2 = w.x * w.x + w.y * w.y + w.z * w.z, th = std::sqrt(t2);
    double a, b;
    if (th < 1e-4) {
        a = 1.0 - t2 / 6.0 + t2 * t2 / 120.0;
        b = 0.5 - t2 / 24.0 + t2 * t2 / 720.0;
    } else {
        a = std::sin(th) / th;
        b = (1.0 - std::cos(th)) / t2;
    }
    const double K[9] = {0.0, -w.z, w.y, w.z, 0.0, -w.x, -w.y, w.x, 0.0};
    double K2[9];
    mm(K, K, K2);
    for (int e = 0; e < 9; ++e) R[e] = ((e % 4) == 0 ? 1.0 : 0.0) + a * K[e] + b * K2[e];
}

// log of a rotation matrix: unit quaternion (largest-component extraction), w >= 0, then the
// rotation vector 2 atan2(|q_v|, q_w) q_v / |q_v| (series below 1e-4 rad)
V3 matrix_to_rotvec(const double* R) {
    const double tr = R[0] + R[4] + R[8];
    double q[4];   // x y z w
    if (tr >= R[0] && tr >= R[4] && tr >= R[8]) {
        q[3] = 1.0 + tr;
        q[0] = R[7] - R[5];
        q[1] = R[2] - R[6];
        q[2] = R[3] - R[1];
    } else {
        const int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        q[i] = 1.0 - tr + 2.0 * R[4 * i];
        q[j] = R[3 * j + i] + R[3 * i + j];
        q[k] = R[3 * k + i] + R[3 * i + k];
        q[3] = R[3 * k + j] - R[3 * j + k];
    }
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double& c : q) c /= n;
    if (q[3] < 0.0)
        for (double& c : q) c = -c;
    const double s = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    const double angle = 2.0 * std::atan2(s, q[3]);
    const double a2 = angle * angle;
    const double scale = angle < 1e-4 ? 2.0 + a2 / 12.0 + 7.0 * a2 * a2 / 2880.0 : angle / std::sin(angle / 2.0);
    return {scale * q[0], scale * q[1], scale * q[2]};
}

// 6x6 helpers (row-major): Cholesky (false unless positive definite), solve, inverse
bool chol6(const double* A, double* L) {
    std::memset(L, 0, 36 * sizeof(double));
    for (int j = 0; j < 6; ++j) {
        double d = A[6 * j + j];
        for (int k = 0; k < j; ++k) d -= L[6 * j + k] * L[6 * j + k];
        if (!(d > 0.0)) return false;
        L[6 * j + j] = std::sqrt(d);
        for (int i = j + 1; i < 6; ++i) {
            double v = A[6 * i + j];
            for (int k = 0; k < j; ++k) v -= L[6 * i + k] * L[6 * j + k];
            L[6 * i + j] = v / L[6 * j + j];
        }
    }
    return true;
}
void chol6_solve(const double* L, const double* b, double* x) {
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= L[6 * i + k] * y[k];
        y[i] = v / L[6 * i + i];
    }
    for (int i = 5; i >= 0; --i) {
        double v = y[i];
        for (int k = i + 1; k < 6; ++k) v -= L[6 * k + i] * x[k];
        x[i] = v / L[6 * i + i];
    }
}
void chol6_inverse(const double* L, double* out) {
    for (int c = 0; c < 6; ++c) {
        double e[6] = {0, 0, 0, 0, 0, 0}, x[6];
        e[c] = 1.0;
        chol6_solve(L, e, x);
        for (int r = 0; r < 6; ++r) out[6 * r + c] = x[r];
    }
}
// general 6x6 inverse by Gauss-Jordan with partial pivoting (false when singular)
bool inv6(const double* A, double* out) {
    double M[6][12];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 12; ++j) M[i][j] = j < 6 ? A[6 * i + j] : (j - 6 == i ? 1.0 : 0.0);
    for (int c = 0; c < 6; ++c) {
        int p = c;
        for (int r = c + 1; r < 6; ++r)
            if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
        if (M[p][c] == 0.0) return false;
        if (p != c)
            for (int j = 0; j < 12; ++j) std::swap(M[p][j], M[c][j]);
        const double iv = 1.0 / M[c][c];
        for (int j = 0; j < 12; ++j) M[c][j] *= iv;
        for (int r = 0; r < 6; ++r) {
            if (r == c || M[r][c] == 0.0) continue;
            const double f = M[r][c];
            for (int j = 0; j < 12; ++j) M[r][j] -= f * M[c][j];
        }
    }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) out[6 * i + j] = M[i][6 + j];
    return true;
}

}   // namespace

struct tslam_imu {
    double Ri[9];
    double na, rw, ng, rwg;
    double rot_floor2, floor2, vis_floor;
    double v0_var, ba0_var, bg0_var;
    double r[3];
    double g[3];
    int accel;
    int ready;
    tslam_imu_state st;
};

static void default_state(tslam_imu_state* s) {
    std::memset(s, 0, sizeof *s);
    s->R[0] = s->R[4] = s->R[8] = 1.0;
    s->var_v = 1.0;
    s->var_b = 0.0025;
    s->var_g = 1e-4;
}

extern "C" {

int tslam_imu_create(const double* rect_R_imu, const double* noise, const double* lever, int accel, tslam_imu** out) {
    if (!rect_R_imu || !noise || !out) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_create: null argument");
    for (int i = 0; i < TSLAM_IMU_NOISE; ++i)
        if (!(noise[i] >= 0.0)) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_create: noise terms must be >= 0");
    auto* f = new tslam_imu{};
    std::memcpy(f->Ri, rect_R_imu, sizeof f->Ri);
    f->ng = noise[0];
    f->rwg = noise[1];
    f->na = noise[2];
    f->rw = noise[3];
    f->rot_floor2 = noise[4] * noise[4];
    f->floor2 = noise[5] * noise[5];
    f->v0_var = noise[6] * noise[6];
    f->ba0_var = noise[7] * noise[7];
    f->bg0_var = noise[8] * noise[8];
    f->vis_floor = noise[9];
    for (int i = 0; i < 3; ++i) f->r[i] = lever ? lever[i] : 0.0;
    f->accel = accel ? 1 : 0;
    default_state(&f->st);
    *out = f;
    return TSLAM_OK;
}

void tslam_imu_destroy(tslam_imu* f) { delete f; }

int tslam_imu_reset(tslam_imu* f) {
    if (!f) return tslam_internal_fail(TSLAM_EINVAL, "null filter");
    f->ready = 0;
    std::memset(f->g, 0, sizeof f->g);
    default_state(&f->st);
    return TSLAM_OK;
}

int tslam_imu_begin(tslam_imu* f, const double* accel) {
    if (!f) return tslam_internal_fail(TSLAM_EINVAL, "null filter");
    std::memset(f->g, 0, sizeof f->g);
    if (f->accel) {   // at rest: the specific force is gravity's reaction
        if (!accel) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_begin: the accelerometer filter needs a sample");
        const V3 s = mv(f->Ri, v3(accel));
        const double n = norm(s);
        if (!(n > 0.0)) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_begin: zero specific force");
        put(-kGravity * s / n, f->g);
    }
    default_state(&f->st);
    f->st.var_v = f->v0_var;
    f->st.var_b = f->ba0_var;
    f->st.var_g = f->bg0_var;
    f->ready = 1;
    return TSLAM_OK;
}

int tslam_imu_ready(const tslam_imu* f) { return f && f->ready ? 1 : 0; }

int tslam_imu_get_state(const tslam_imu* f, tslam_imu_state* st) {
    if (!f || !st) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    *st = f->st;
    return TSLAM_OK;
}

int tslam_imu_set_state(tslam_imu* f, const tslam_imu_state* st) {
    if (!f || !st) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    f->st = *st;
    return TSLAM_OK;
}

int tslam_imu_predict(const tslam_imu* f, const tslam_imu_state* st, double dt, const double* gyro, const double* accel,
                   tslam_imu_step* out) {
    if (!f || !st || !gyro || !out) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    if (!(dt > 0.0)) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_predict: dt must be > 0");
    if (f->accel && !accel) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_predict: the accelerometer filter needs a sample");
    tslam_imu_step s{};
    s.dt = dt;
    std::memcpy(s.gyro, gyro, sizeof s.gyro);
    const V3 w = mv(f->Ri, v3(gyro) - v3(st->bg));
    put(w, s.w);
    rotvec_to_matrix(neg(w) * dt, s.R_rel);
    s.w_rot = 1.0 / (f->ng * f->ng * dt + st->var_g * dt * dt + f->rot_floor2);
    if (!f->accel) {
        *out = s;
        return TSLAM_OK;
    }
    const V3 alpha = st->has_w_prev ? (w - v3(st->w_prev)) / dt : V3{0.0, 0.0, 0.0};
    const V3 w_w = mv(st->R, w), al_w = mv(st->R, alpha), r_w = mv(st->R, v3(f->r));
    const V3 a_w = ((mv(st->R, mv(f->Ri, v3(accel) - v3(st->ba))) + v3(f->g)) - cross(w_w, cross(w_w, r_w))) - cross(al_w, r_w);
    const V3 centre = mtv(st->R, v3(st->v) * dt + (0.5 * a_w) * dt * dt);   // new camera centre, old axes
    const double var_t = ((st->var_v * (dt * dt) + f->na * f->na * (dt * dt * dt) / 3.0) +
                          st->var_b * (dt * dt * dt * dt) / 4.0) + f->floor2;
    put(neg(mv(s.R_rel, centre)), s.t_rel);
    s.w_trans = 1.0 / var_t;
    put(v3(st->v) + a_w * dt, s.v1);
    s.var_v1 = (st->var_v + f->na * f->na * dt) + st->var_b * dt * dt;
    s.has_v1 = 1;
    *out = s;
    return TSLAM_OK;
}

int tslam_imu_coast(const tslam_imu* f, const tslam_imu_state* st, const tslam_imu_step* s, tslam_imu_state* out) {
    if (!f || !st || !s || !out) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    tslam_imu_state n = *st;
    mmt(st->R, s->R_rel, n.R);
    n.var_g = st->var_g + f->rwg * f->rwg * s->dt;
    std::memcpy(n.w_prev, s->w, sizeof n.w_prev);
    n.has_w_prev = 1;
    if (f->accel) {
        std::memcpy(n.v, s->v1, sizeof n.v);
        n.var_v = s->var_v1;
        n.var_b = st->var_b + f->rw * f->rw * s->dt;
    }
    *out = n;
    return TSLAM_OK;
}

int tslam_imu_correct(const tslam_imu* f, const tslam_imu_state* st, const tslam_imu_step* s, const double* t_rel,
                      const double* cov, tslam_imu_state* out) {
    if (!f || !st || !s || !t_rel || !cov || !out) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    const double dt = s->dt;
    const double rv[9] = {t_rel[0], t_rel[1], t_rel[2], t_rel[4], t_rel[5], t_rel[6], t_rel[8], t_rel[9], t_rel[10]};
    const V3 tv = {t_rel[3], t_rel[7], t_rel[11]};
    // gyroscope bias: the rate the vision saw against the sample
    const double var_g1 = st->var_g + f->rwg * f->rwg * dt;
    const V3 w_v = neg(matrix_to_rotvec(rv)) / dt;
    const V3 z = v3(s->gyro) - mtv(f->Ri, w_v);
    const double var_z = ((cov[21] + cov[28]) + cov[35]) / 3.0 / (dt * dt) + f->ng * f->ng / dt +
                         (f->vis_floor / dt) * (f->vis_floor / dt);
    const double kg = var_g1 / (var_g1 + var_z);
    tslam_imu_state n = *st;
    mmt(st->R, rv, n.R);
    put(v3(st->bg) + kg * (z - v3(st->bg)), n.bg);
    n.var_g = (1.0 - kg) * var_g1;
    std::memcpy(n.w_prev, s->w, sizeof n.w_prev);
    n.has_w_prev = 1;
    if (f->accel) {   // velocity and accelerometer bias towards the visual motion
        const V3 v_vis = mv(st->R, neg(mtv(rv, tv))) / dt;
        const double var_vis = ((cov[0] + cov[7]) + cov[14]) / 3.0 / (dt * dt);
        const V3 innov = v_vis - v3(s->v1);
        const double k = s->var_v1 / (s->var_v1 + var_vis);
        const double var_b1 = st->var_b + f->rw * f->rw * dt;
        const double kb = var_b1 / ((var_b1 + (var_vis + s->var_v1) / (dt * dt)) + f->na * f->na / dt);
        const V3 e_imu = mtv(f->Ri, mtv(st->R, innov / dt));
        put(v3(s->v1) + k * innov, n.v);
        put(v3(st->ba) - kb * e_imu, n.ba);
        n.var_v = (1.0 - k) * s->var_v1;
        n.var_b = (1.0 - kb) * var_b1;
    }
    *out = n;
    return TSLAM_OK;
}

int tslam_imu_batch_priors(const tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                           tslam_imu_step* out, int32_t* valid) {
    if (!f || n < 0 || (n > 0 && (!dt || !gyro || !out || !valid))) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    tslam_imu_state st = f->st;
    for (int k = 0; k < n; ++k) {
        valid[k] = 0;
        if (!std::isfinite(dt[k]) || !f->ready) continue;
        const int rc = tslam_imu_predict(f, &st, dt[k], gyro + 3 * k, accel ? accel + 3 * k : nullptr, &out[k]);
        if (rc != TSLAM_OK) return rc;
        valid[k] = 1;
        tslam_imu_coast(f, &st, &out[k], &st);
    }
    return TSLAM_OK;
}

int tslam_imu_absorb(tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                     const int32_t* status, const double* t_rel, const double* cov) {
    if (!f || n < 0 || (n > 0 && (!dt || !gyro || !status || !t_rel || !cov)))
        return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    for (int k = 0; k < n; ++k) {
        if (!std::isfinite(dt[k]) || !f->ready) continue;
        tslam_imu_step s;
        const int rc = tslam_imu_predict(f, &f->st, dt[k], gyro + 3 * k, accel ? accel + 3 * k : nullptr, &s);
        if (rc != TSLAM_OK) return rc;
        if (status[k] == 0) tslam_imu_correct(f, &f->st, &s, t_rel + 16 * k, cov + 36 * k, &f->st);
        else tslam_imu_coast(f, &f->st, &s, &f->st);
    }
    return TSLAM_OK;
}

int tslam_imu_vision_only(const double* T, const double* cov, double sigma2, const tslam_imu_step* s, double* T_out,
                          double* cov_out) {
    if (!T || !cov || !s || !T_out || !cov_out) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    double Tc[16], Cc[36];
    std::memcpy(Tc, T, sizeof Tc);
    std::memcpy(Cc, cov, sizeof Cc);
    std::memcpy(T_out, Tc, sizeof Tc);
    std::memcpy(cov_out, Cc, sizeof Cc);
    if (!(sigma2 > 0.0) || !(s->w_rot > 0.0 || s->w_trans > 0.0)) return TSLAM_OK;
    double h[36];
    if (!inv6(Cc, h)) return TSLAM_OK;
    double hv[36];
    for (int e = 0; e < 36; ++e) h[e] *= sigma2;
    std::memcpy(hv, h, sizeof hv);
    for (int i = 0; i < 3; ++i) {
        hv[6 * i + i] -= s->w_trans;
        hv[6 * (i + 3) + i + 3] -= s->w_rot;
    }
    double hs[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) hs[6 * i + j] = 0.5 * (hv[6 * i + j] + hv[6 * j + i]);
    double L[36];
    if (!chol6(hs, L)) return TSLAM_OK;   // the vision alone is not positive definite: unchanged
    const double R[9] = {Tc[0], Tc[1], Tc[2], Tc[4], Tc[5], Tc[6], Tc[8], Tc[9], Tc[10]};
    const V3 t = {Tc[3], Tc[7], Tc[11]};
    double a[9];
    mmt(s->R_rel, R, a);
    const V3 delta = 0.5 * V3{a[7] - a[5], a[2] - a[6], a[3] - a[1]};
    const V3 dtr = s->w_trans * (t - v3(s->t_rel)), drot = neg(s->w_rot * delta);
    const double b[6] = {dtr.x, dtr.y, dtr.z, drot.x, drot.y, drot.z};
    double d[6];
    chol6_solve(L, b, d);
    const double w0 = d[3], w1 = d[4], w2 = d[5];
    const double A[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
    double A2[9];
    mm(A, A, A2);
    const double sc = 4.0 / (4.0 + ((w0 * w0 + w1 * w1) + w2 * w2));
    double ru[9];
    for (int e = 0; e < 9; ++e) ru[e] = ((e % 4) == 0 ? 1.0 : 0.0) + sc * (A[e] + 0.5 * A2[e]);
    double Rn[9];
    mm(ru, R, Rn);
    const V3 tn = mv(ru, t) + V3{d[0], d[1], d[2]};
    std::memset(T_out, 0, 16 * sizeof(double));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T_out[4 * i + j] = Rn[3 * i + j];
    T_out[3] = tn.x;
    T_out[7] = tn.y;
    T_out[11] = tn.z;
    T_out[15] = 1.0;
    double hinv[36];
    chol6_inverse(L, hinv);
    for (int e = 0; e < 36; ++e) cov_out[e] = sigma2 * hinv[e];
    return TSLAM_OK;
}

int tslam_imu_gravity(const tslam_imu* f, double* g) {
    if (!f || !g) return tslam_internal_fail(TSLAM_EINVAL, "null argument");
    std::memcpy(g, f->g, sizeof f->g);
    return TSLAM_OK;
}

// Accelerometer preintegration between two keyframes (spec: oracle/numpy_ba.py preintegrate), in
// the first keyframe's camera axes, with the filter's Ri and lever arm: per interval k the rate
// w = Ri (gyro - bg), alpha = (w - w_prev) / dt, the camera's specific force
// a = Ri (accel - ba) - w x (w x r) - alpha x r; dp += dv dt + dR a dt^2 / 2,
// Jp += Jv dt - dR Ri dt^2 / 2, dv += dR a dt, Jv -= dR Ri dt, dR <- dR exp([w dt]x).
// right Jacobian of SO(3) (oracle numpy_ba._jr_so3): I - (1 - cos t) / t^2 [w]x + (t - sin t) / t^3 [w]x^2
static void jr_so3(V3 w, double* J) {
    const double t2 = w.x * w.x + w.y * w.y + w.z * w.z, th = std::sqrt(t2);
    double a, b;
    if (th < 1e-4) {
        a = 0.5;
        b = 1.0 / 6.0;
    } else {
        a = (1.0 - std::cos(th)) / t2;
        b = (th - std::sin(th)) / (t2 * th);
    }
    const double K[9] = {0.0, -w.z, w.y, w.z, 0.0, -w.x, -w.y, w.x, 0.0};
    double K2[9];
    mm(K, K, K2);
    for (int e = 0; e < 9; ++e) J[e] = ((e % 4) == 0 ? 1.0 : 0.0) - a * K[e] + b * K2[e];
}

int tslam_imu_preintegrate(const tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                           const double* bg, const double* ba, const double* w_prev, const double* frame_R_imu,
                           const double* lever, double v_floor, double p_floor, double r_floor, double ba_floor,
                           double bg_floor, double* record) {
    if (!f || n < 1 || !dt || !gyro || !accel || !bg || !ba || !record)
        return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_preintegrate: null argument or n < 1");
    double dR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, Jv[9] = {}, Jp[9] = {}, Jvg[9] = {}, Jpg[9] = {}, JR[9] = {};
    V3 dv{0, 0, 0}, dp{0, 0, 0};
    double T = 0.0;
    bool have_prev = w_prev != nullptr;
    V3 wp = have_prev ? v3(w_prev) : V3{0, 0, 0};
    const double* Ri = frame_R_imu ? frame_R_imu : f->Ri;   // the factor's frame (default: the filter's camera)
    const V3 r = v3(lever ? lever : f->r), bgv = v3(bg), bav = v3(ba);
    double dRRi[9];
    for (int k = 0; k < n; ++k) {
        const double h = dt[k];
        if (!(h > 0.0)) return tslam_internal_fail(TSLAM_EINVAL, "tslam_imu_preintegrate: dt must be > 0");
        const V3 w = mv(Ri, v3(gyro + 3 * k) - bgv);
        const V3 al = have_prev ? (w - wp) / h : V3{0, 0, 0};
        const V3 a = mv(Ri, v3(accel + 3 * k) - bav) - cross(w, cross(w, r)) - cross(al, r);
        const V3 Ra = mv(dR, a);
        mm(dR, Ri, dRRi);
        // dR [a]x JR: the gyroscope bias's first-order effect on the specific force's rotation
        const double Ka[9] = {0.0, -a.z, a.y, a.z, 0.0, -a.x, -a.y, a.x, 0.0};
        double KJ[9], RaJ[9];
        mm(Ka, JR, KJ);
        mm(dR, KJ, RaJ);
        dp = dp + dv * h + 0.5 * Ra * h * h;
        for (int e = 0; e < 9; ++e) Jp[e] = Jp[e] + Jv[e] * h - 0.5 * dRRi[e] * h * h;
        for (int e = 0; e < 9; ++e) Jpg[e] = Jpg[e] + Jvg[e] * h - 0.5 * RaJ[e] * h * h;
        dv = dv + Ra * h;
        for (int e = 0; e < 9; ++e) Jv[e] = Jv[e] - dRRi[e] * h;
        for (int e = 0; e < 9; ++e) Jvg[e] = Jvg[e] - RaJ[e] * h;
        double E[9], nR[9], Jr[9], JrRi[9], nJ[9];
        rotvec_to_matrix(w * h, E);
        jr_so3(w * h, Jr);
        mm(Jr, Ri, JrRi);
        for (int i = 0; i < 3; ++i)   // JR <- E^T JR - Jr Ri h
            for (int j = 0; j < 3; ++j)
                nJ[3 * i + j] = (E[i] * JR[j] + E[3 + i] * JR[3 + j] + E[6 + i] * JR[6 + j]) - JrRi[3 * i + j] * h;
        std::memcpy(JR, nJ, sizeof JR);
        mm(dR, E, nR);
        std::memcpy(dR, nR, sizeof dR);
        T += h;
        wp = w;
        have_prev = true;
    }
    std::memset(record, 0, TSLAM_BA_INE_RECORD * sizeof(double));
    put(dv, record);
    put(dp, record + 3);
    std::memcpy(record + 6, Jv, sizeof Jv);
    std::memcpy(record + 15, Jp, sizeof Jp);
    put(bav, record + 24);
    record[27] = T;
    record[28] = 1.0 / (f->na * f->na * T + v_floor * v_floor);
    record[29] = 1.0 / (f->na * f->na * T * T * T / 3.0 + p_floor * p_floor);
    record[30] = f->ng > 0.0 ? 1.0 / (f->ng * f->ng * T + r_floor * r_floor) : 0.0;
    record[31] = f->rw > 0.0 ? 1.0 / (f->rw * f->rw * T + ba_floor * ba_floor) : 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) record[32 + 3 * i + j] = dR[3 * j + i];   // M = dR^T
    mm(dR, JR, record + 41);                                                  // JRe = dR JR
    std::memcpy(record + 50, Jvg, sizeof Jvg);
    std::memcpy(record + 59, Jpg, sizeof Jpg);
    put(bgv, record + 68);
    record[71] = f->rwg > 0.0 ? 1.0 / (f->rwg * f->rwg * T + bg_floor * bg_floor) : 0.0;
    return TSLAM_OK;
}

}   // extern "C"
