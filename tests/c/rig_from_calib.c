/* Native caller of the C-ABI (tests/test_native_calib.py, tests/test_gpu_native_rig.py): the
 * binding a C/C++ host of the reference's camera pipeline would write against include/tslam.h.
 *
 *   rig_from_calib maps <calib.txt> <out.bin>
 *       per pair found by tslam_rig_pairs: int32 left, right; tslam_rectify_pair's desc scalars
 *       (fx fy cx cy baseline as f64), base_T_rect[16] f64, map_left and map_right (H*W*2 int32)
 *   rig_from_calib run <calib.txt> <params.bin> <frames.bin> <n_frames> <batch> <out.bin>
 *       tslam_create_rig, then the frames through tslam_submit_host in batches of <batch> with
 *       timestamps 0.05*i, every batch drained with tslam_poll_batch(block = 1); writes per frame
 *       T_abs[P][16] f64, stats[P][8] int32, and the rig's T_abs[16] when P > 1, then the
 *       last tslam_poll_pose (T[16], cov[36], ts f64, state int32, conf f32).
 *
 * calib.txt: one camera per line, "source cam_idx width height n_coeffs K[9] D[14] T[16]"
 * (doubles printed with 17 significant digits, so they read back exactly). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tslam.h"

#define MAX_CAMS 16

static char names[MAX_CAMS][64];

static int read_calib(const char* path, tslam_camera_desc* cams) {
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int n = 0;
    while (n < MAX_CAMS) {
        tslam_camera_desc* c = &cams[n];
        memset(c, 0, sizeof(*c));
        if (fscanf(f, "%63s %d %d %d %d", names[n], &c->cam_idx, &c->width, &c->height, &c->n_coeffs) != 5) break;
        int ok = 1;
        for (int i = 0; i < 9; ++i) ok &= fscanf(f, "%lf", &c->K[i]) == 1;
        for (int i = 0; i < 14; ++i) ok &= fscanf(f, "%lf", &c->D[i]) == 1;
        for (int i = 0; i < 16; ++i) ok &= fscanf(f, "%lf", &c->world_T_cam[i]) == 1;
        if (!ok) {
            fclose(f);
            return -1;
        }
        c->source = names[n];
        ++n;
    }
    fclose(f);
    return n;
}

static int die(const char* what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, tslam_last_error());
    return 1;
}

static int cmd_maps(const tslam_camera_desc* cams, int n, const char* out_path) {
    int32_t pairs[2 * MAX_CAMS];
    const int np = tslam_rig_pairs(cams, n, pairs, MAX_CAMS);
    if (np < 0) return die("tslam_rig_pairs", np);
    FILE* out = fopen(out_path, "wb");
    if (!out) return 1;
    for (int p = 0; p < np; ++p) {
        const tslam_camera_desc* l = &cams[pairs[2 * p]];
        const size_t cells = (size_t)l->width * l->height * 2;
        int32_t* ml = malloc(cells * sizeof(int32_t));
        int32_t* mr = malloc(cells * sizeof(int32_t));
        double base[16];
        tslam_stereo_desc d;
        const int rc = tslam_rectify_pair(l, &cams[pairs[2 * p + 1]], &d, ml, mr, base, NULL);
        if (rc) return die("tslam_rectify_pair", rc);
        const double sc[5] = {d.fx, d.fy, d.cx, d.cy, d.baseline};
        fwrite(&pairs[2 * p], sizeof(int32_t), 2, out);
        fwrite(sc, sizeof(double), 5, out);
        fwrite(base, sizeof(double), 16, out);
        fwrite(ml, sizeof(int32_t), cells, out);
        fwrite(mr, sizeof(int32_t), cells, out);
        free(ml);
        free(mr);
    }
    fclose(out);
    return 0;
}

static void* read_file(const char* path, size_t* size) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *size = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void* buf = malloc(*size);
    if (fread(buf, 1, *size, f) != *size) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    return buf;
}

static int cmd_run(const tslam_camera_desc* cams, int n, const char* params_path, const char* frames_path, int n_frames,
                   int batch, const char* out_path) {
    size_t psize = 0, fsize = 0;
    tslam_params* params = read_file(params_path, &psize);
    uint8_t* frames = read_file(frames_path, &fsize);
    if (!params || psize != sizeof(tslam_params) || !frames) {
        fprintf(stderr, "bad params / frames file\n");
        return 1;
    }
    tslam_handle* h = NULL;
    int rc = tslam_create_rig(cams, n, params, 0, &h);
    if (rc) return die("tslam_create_rig", rc);
    const int np = tslam_rig_pairs(cams, n, NULL, 0);
    const size_t frame_bytes = fsize / (size_t)n_frames;
    double* T_abs = malloc(sizeof(double) * 16 * np * batch);
    int32_t* stats = malloc(sizeof(int32_t) * 8 * np * batch);
    double* rig_T = malloc(sizeof(double) * 16 * batch);
    double* ts = malloc(sizeof(double) * batch);
    FILE* out = fopen(out_path, "wb");
    for (int f0 = 0; f0 < n_frames; f0 += batch) {
        const int nb = n_frames - f0 < batch ? n_frames - f0 : batch;
        for (int i = 0; i < nb; ++i) ts[i] = 0.05 * (f0 + i);
        if ((rc = tslam_submit_host(h, frames + frame_bytes * f0, ts, nb))) return die("tslam_submit_host", rc);
        int64_t first = -1;
        int got = 0;
        rc = tslam_poll_batch(h, 1, batch, NULL, T_abs, NULL, stats, NULL, np > 1 ? rig_T : NULL, NULL, NULL, ts, &first, &got);
        if (rc != 1 || got != nb || first != f0) {
            fprintf(stderr, "poll_batch rc=%d got=%d first=%lld: %s\n", rc, got, (long long)first, tslam_last_error());
            return 1;
        }
        for (int i = 0; i < nb; ++i) {
            fwrite(T_abs + (size_t)16 * np * i, sizeof(double), 16 * np, out);
            fwrite(stats + (size_t)8 * np * i, sizeof(int32_t), 8 * np, out);
            if (np > 1) fwrite(rig_T + 16 * i, sizeof(double), 16, out);
        }
    }
    double T[16], cov[36], t = 0;
    int32_t state = -1;
    float conf = -1;
    rc = tslam_poll_pose(h, T, cov, &t, &state, &conf);
    if (rc < 0) return die("tslam_poll_pose", rc);
    fwrite(T, sizeof(double), 16, out);
    fwrite(cov, sizeof(double), 36, out);
    fwrite(&t, sizeof(double), 1, out);
    fwrite(&state, sizeof(int32_t), 1, out);
    fwrite(&conf, sizeof(float), 1, out);
    fclose(out);
    tslam_destroy(h);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s maps|run <calib.txt> ...\n", argv[0]);
        return 2;
    }
    tslam_camera_desc cams[MAX_CAMS];
    const int n = read_calib(argv[2], cams);
    if (n <= 0) {
        fprintf(stderr, "no cameras in %s\n", argv[2]);
        return 1;
    }
    if (!strcmp(argv[1], "maps")) return cmd_maps(cams, n, argv[3]);
    if (!strcmp(argv[1], "run") && argc == 8) return cmd_run(cams, n, argv[3], argv[4], atoi(argv[5]), atoi(argv[6]), argv[7]);
    fprintf(stderr, "bad command\n");
    return 2;
}
