// k_dense.hip — dense-map outputs of the TSDF volume (after integration):
// the marching-cubes surface mesh and the exact, capped Euclidean signed distance field nvblox
// publishes (launch/thor_nvblox.launch.py:21-103).  Spec: thor_slam_amd/dense.py; CPU restatement:
// oracle/numpy_dense.py.  Volumes are the k_tsdf.hip grid: tsdf / weight f32 [nz][ny][nx].
//
// Mesh, three launches (no host round trip between them):
//   k_mesh_count  thread per cube (x fastest): the 8 corners' weights and signs -> the cube's
//                 configuration byte (0 when unobserved) and the block's triangle total;
//   k_mesh_scan   one block: exclusive scan of the block totals -> each block's first triangle,
//                 and the mesh's triangle count;
//   k_mesh_emit   thread per cube again: block-local exclusive scan of the counts, the triangles'
//                 vertices interpolated on the crossing edges (f32, edge values read from the
//                 edge's lower voxel so both cubes of a shared edge produce the same vertex),
//                 9 f32 per triangle in cube order (+ 9 f32 of vertex colours with the colour
//                 layer: each vertex takes its edge's nearer voxel's colour).
//   Roofline: HBM — the 2 x 4 B of every voxel read once per pass (neighbour corners hit L2), plus
//   1 B of configuration per cube and 36 B per triangle.
//
// ESDF, windowed exact distance transform (integer squared voxel distances; R = floor(max / s)):
//   k_esdf_sites    site (observed, |tsdf| <= site) -> 0, else the cap R^2 + 1 (int32);
//   k_edt_pass_x_lds / k_edt_pass_yz_lds (R <= 64; k_edt_pass beyond): along one axis,
//                   g'(x) = min_{|d| <= R} g(x + d) + d^2, capped — x, then y, then z (exact for every
//                   distance <= R voxels); each block stages its line segments plus the R halo in
//                   LDS once and the (2R + 1)-tap minimum runs on LDS reads;
//   k_esdf_finish   sign (tsdf < 0 and not a site), s sqrt(d^2) from the host-built f32 table,
//                   +-max beyond R, NaN where unobserved.
//   The 2-D slice runs k_esdf_slice_sites (a column is a site / observed when any voxel of the
//   height band is) and the x and z passes on the [nz][nx] plane.
//   Roofline: LDS / VALU — (2R + 1) LDS reads per voxel and pass; HBM reads the tile + halo once.
#include "tslam_common.h"
#include "tslam_mc_table.h"

#define DENSE_THREADS 256

// --- mesh ---------------------------------------------------------------------------------------

struct CubeAt {
    int i, j, k;
    int64_t v;   // base voxel
};

__device__ __forceinline__ CubeAt cube_at(const DenseArgs& a, uint32_t q) {
    const uint32_t cx = (uint32_t)(a.nx - 1), cy = (uint32_t)(a.ny - 1);
    CubeAt c;
    c.i = (int)(q % cx);
    const uint32_t r = q / cx;
    c.j = (int)(r % cy);
    c.k = (int)(r / cy);
    c.v = ((int64_t)c.k * a.ny + c.j) * a.nx + c.i;
    return c;
}

// configuration byte of cube q (0 when a corner is unobserved)
__device__ __forceinline__ uint32_t cube_config(const DenseArgs& a, const CubeAt& c) {
    const int64_t sy = a.nx, sz = (int64_t)a.nx * a.ny;
    uint32_t cfg = 0;
    bool obs = true;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const int64_t o = c.v + (n & 1) + ((n >> 1) & 1) * sy + ((n >> 2) & 1) * sz;
        obs &= a.weight[o] >= a.min_weight;
        cfg |= (a.tsdf[o] < 0.0f ? 1u : 0u) << n;
    }
    return obs ? cfg : 0u;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* s_w) {
    v = (uint32_t)wave_sum_i32((int)v);
    if (wave_lane() == 0) s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
    for (int w = 0; w < DENSE_THREADS / 64; ++w) t += s_w[w];
    return t;
}

__global__ __launch_bounds__(DENSE_THREADS) void k_mesh_count(DenseArgs a, uint8_t* cfg_out, uint32_t* block_sums) {
    __shared__ uint32_t s_w[DENSE_THREADS / 64];
    const uint32_t q = blockIdx.x * DENSE_THREADS + threadIdx.x;
    uint32_t n = 0;
    if (q < a.n_cubes) {
        const uint32_t cfg = cube_config(a, cube_at(a, q));
        cfg_out[q] = (uint8_t)cfg;
        n = TSLAM_MC_COUNT[cfg];
    }
    const uint32_t t = block_sum_u32(n, s_w);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = t;
}

// One block of 1024 threads: block_off[b] = sum of block_sums[0..b), *total = the sum of all.
__global__ __launch_bounds__(1024) void k_mesh_scan(const uint32_t* block_sums, int nb, uint64_t* block_off,
                                                    uint64_t* total) {
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c0 = 0; c0 < nb; c0 += 1024) {
        const int b = c0 + threadIdx.x;
        const uint64_t x = b < nb ? block_sums[b] : 0;
        uint64_t inc = x;   // wave inclusive scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint64_t before = s_carry;
        for (int k = 0; k < w; ++k) before += s_w[k];
        if (b < nb) block_off[b] = before + inc - x;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = before + inc;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = s_carry;
}

__global__ __launch_bounds__(DENSE_THREADS) void k_mesh_emit(DenseArgs a, const uint8_t* cfg_in, const uint64_t* block_off,
                                                             float* tris, float* cols, int64_t cap) {
    __shared__ uint32_t s_w[DENSE_THREADS / 64];
    const uint32_t q = blockIdx.x * DENSE_THREADS + threadIdx.x;
    const uint32_t cfg = q < a.n_cubes ? cfg_in[q] : 0u;
    const uint32_t n = TSLAM_MC_COUNT[cfg];
    // block-local exclusive scan of the counts
    const int lane = wave_lane(), w = threadIdx.x >> 6;
    uint32_t inc = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (int k = 0; k < w; ++k) before += s_w[k];
    if (n == 0) return;
    const CubeAt c = cube_at(a, q);
    const int64_t first = (int64_t)block_off[blockIdx.x] + before + inc - n;
    const int64_t stride[3] = {1, a.nx, (int64_t)a.nx * a.ny};
    for (uint32_t t = 0; t < n; ++t) {
        const int64_t tri = first + t;
        if (tri >= cap) return;
        float* out = tris + tri * 9;
        for (int vtx = 0; vtx < 3; ++vtx) {
            const int e = TSLAM_MC_TRIS[(cfg * TSLAM_MC_MAX_TRIS + t) * 3 + vtx];
            const int ax = e >> 2, m = e & 3;
            const int o0 = ax == 0 ? 1 : 0, o1 = ax == 2 ? 1 : 2;   // the other two axes, low first
            int off[3] = {0, 0, 0};
            off[o0] = m & 1;
            off[o1] = m >> 1;
            const int64_t vb = c.v + off[0] * stride[0] + off[1] * stride[1] + off[2] * stride[2];
            const float va = a.tsdf[vb], ve = a.tsdf[vb + stride[ax]];
            const float tt = va / (va - ve);   // IEEE f32 division (no fast-math, no contraction)
            float p[3];
            p[0] = (float)(a.ox + a.s * ((c.i + off[0]) + 0.5));
            p[1] = (float)(a.oy + a.s * ((c.j + off[1]) + 0.5));
            p[2] = (float)(a.oz + a.s * ((c.k + off[2]) + 0.5));
            p[ax] = p[ax] + tt * a.sf;
            out[3 * vtx + 0] = p[0];
            out[3 * vtx + 1] = p[1];
            out[3 * vtx + 2] = p[2];
            if (a.color) {   // the colour of the edge's voxel nearer to the vertex
                const float* cv = a.color + 3 * (tt < 0.5f ? vb : vb + stride[ax]);
                float* oc = cols + tri * 9 + 3 * vtx;
                oc[0] = cv[0];
                oc[1] = cv[1];
                oc[2] = cv[2];
            }
        }
    }
}

// --- ESDF ---------------------------------------------------------------------------------------

__global__ __launch_bounds__(DENSE_THREADS) void k_esdf_sites(DenseArgs a, int32_t* g) {
    const int64_t v = (int64_t)blockIdx.x * DENSE_THREADS + threadIdx.x;
    if (v >= a.n_voxels) return;
    const bool site = a.weight[v] >= a.min_weight && fabsf(a.tsdf[v]) <= a.site_dist;
    g[v] = site ? 0 : a.cap;
}

// columns (i, k) of the band y0 <= j < y1: g [nz][nx] and the observed flag
__global__ __launch_bounds__(DENSE_THREADS) void k_esdf_slice_sites(DenseArgs a, int y0, int y1, int32_t* g, uint8_t* obs) {
    const int64_t c = (int64_t)blockIdx.x * DENSE_THREADS + threadIdx.x;
    if (c >= (int64_t)a.nx * a.nz) return;
    const int64_t i = c % a.nx, k = c / a.nx;
    bool site = false, seen = false;
    for (int j = y0; j < y1; ++j) {
        const int64_t v = ((int64_t)k * a.ny + j) * a.nx + i;
        const bool o = a.weight[v] >= a.min_weight;
        seen |= o;
        site |= o && fabsf(a.tsdf[v]) <= a.site_dist;
    }
    g[c] = site ? 0 : a.cap;
    obs[c] = seen ? 1 : 0;
}

// g_out[v] = min(cap, min_{|d| <= R, 0 <= x + d < n} g_in[v + d stride] + d^2), x = (v / stride) % n
__global__ __launch_bounds__(DENSE_THREADS) void k_edt_pass(const int32_t* g_in, int32_t* g_out, int64_t total, int n,
                                                            int64_t stride, int R, int32_t cap) {
    const int64_t v = (int64_t)blockIdx.x * DENSE_THREADS + threadIdx.x;
    if (v >= total) return;
    const int x = (int)((v / stride) % n);
    const int lo = max(-R, -x), hi = min(R, n - 1 - x);
    int32_t best = g_in[v];
    for (int d = lo; d <= hi; ++d) {
        const int32_t cand = g_in[v + d * stride] + d * d;
        best = cand < best ? cand : best;
    }
    g_out[v] = best < cap ? best : cap;
}

// The same pass staged through LDS, for R <= EDT_LDS_R (the usual 2 m / 5 cm = 40): every value a
// block needs is read from HBM / L2 once into LDS and the (2R + 1)-tap minimum runs on LDS reads.
//   x (stride 1): block = 256 consecutive voxels of one row, LDS = [x0 - R, x0 + 256 + R);
//   y / z: block = 64 consecutive x columns x EDT_TA outputs along the axis, LDS = (EDT_TA + 2R)
//   rows of 64 values; thread (column, quarter) computes EDT_TA / 4 outputs.
#define EDT_LDS_R 64
#define EDT_TA 64
__global__ __launch_bounds__(DENSE_THREADS) void k_edt_pass_x_lds(const int32_t* g_in, int32_t* g_out, int nx,
                                                                  int64_t rows, int R, int32_t cap) {
    __shared__ int32_t s_g[DENSE_THREADS + 2 * EDT_LDS_R];
    const int tiles = (nx + DENSE_THREADS - 1) / DENSE_THREADS;
    const int64_t row = blockIdx.x / tiles;
    const int x0 = (int)(blockIdx.x - row * tiles) * DENSE_THREADS;
    const int32_t* in = g_in + row * nx;
    for (int i = threadIdx.x; i < DENSE_THREADS + 2 * R; i += DENSE_THREADS) {
        const int x = x0 - R + i;
        s_g[i] = (x >= 0 && x < nx) ? in[x] : cap;   // outside the row: no site (cap never wins)
    }
    __syncthreads();
    const int x = x0 + (int)threadIdx.x;
    if (x >= nx) return;
    const int32_t* c = s_g + threadIdx.x + R;
    int32_t best = c[0];
    for (int d = 1; d <= R; ++d) {
        const int32_t dd = d * d;
        best = min(best, min(c[-d], c[d]) + dd);
    }
    g_out[row * nx + x] = min(best, cap);
}

// y or z: `n` = extent along the axis, `stride` = its voxel stride, `nx` = the x extent (columns
// of 64 are x-contiguous), `outer` = the count of independent planes (z for the y pass, 1 plane
// of nx * ny columns for the z pass is handled by treating x as nx * ny).
__global__ __launch_bounds__(DENSE_THREADS) void k_edt_pass_yz_lds(const int32_t* g_in, int32_t* g_out, int ncol,
                                                                   int n, int64_t stride, int64_t plane, int R,
                                                                   int32_t cap) {
    extern __shared__ int32_t s_t[];   // [(EDT_TA + 2R)][64]
    const int cgroups = (ncol + 63) / 64, agroups = (n + EDT_TA - 1) / EDT_TA;
    int64_t b = blockIdx.x;
    const int cg = (int)(b % cgroups);
    b /= cgroups;
    const int ag = (int)(b % agroups);
    const int64_t p = b / agroups;                 // plane index
    const int col0 = cg * 64, a0 = ag * EDT_TA;
    const int lane = threadIdx.x & 63, quarter = threadIdx.x >> 6;
    const int col = col0 + lane;
    const int32_t* in = g_in + p * plane + col;
    const int span = EDT_TA + 2 * R;
    for (int r = quarter; r < span; r += 4) {
        const int a = a0 - R + r;
        s_t[r * 64 + lane] = (col < ncol && a >= 0 && a < n) ? in[(int64_t)a * stride] : cap;
    }
    __syncthreads();
    if (col >= ncol) return;
    for (int o = quarter; o < EDT_TA; o += 4) {
        const int a = a0 + o;
        if (a >= n) break;
        const int32_t* c = s_t + (o + R) * 64 + lane;
        int32_t best = c[0];
        for (int d = 1; d <= R; ++d) {
            const int32_t dd = d * d;
            best = min(best, min(c[-d * 64], c[d * 64]) + dd);
        }
        g_out[p * plane + (int64_t)a * stride + col] = min(best, cap);
    }
}

__global__ __launch_bounds__(DENSE_THREADS) void k_esdf_finish(DenseArgs a, const int32_t* g, const float* tab, float* out) {
    const int64_t v = (int64_t)blockIdx.x * DENSE_THREADS + threadIdx.x;
    if (v >= a.n_voxels) return;
    const float w = a.weight[v], t = a.tsdf[v];
    const int32_t d2 = g[v];
    float d = d2 >= a.cap ? a.max_dist : tab[d2];
    if (t < 0.0f && d2 > 0) d = -d;
    out[v] = w >= a.min_weight ? d : __builtin_nanf("");
}

__global__ __launch_bounds__(DENSE_THREADS) void k_esdf_slice_finish(DenseArgs a, const int32_t* g, const uint8_t* obs,
                                                                     const float* tab, float* out) {
    const int64_t c = (int64_t)blockIdx.x * DENSE_THREADS + threadIdx.x;
    if (c >= (int64_t)a.nx * a.nz) return;
    const int32_t d2 = g[c];
    out[c] = obs[c] ? (d2 >= a.cap ? a.max_dist : tab[d2]) : __builtin_nanf("");
}

// --- launchers ----------------------------------------------------------------------------------

static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + DENSE_THREADS - 1) / DENSE_THREADS); }

void launch_mesh_count(const DenseArgs& a, uint8_t* cfg, uint32_t* block_sums, uint64_t* block_off, uint64_t* total,
                       hipStream_t s) {
    const unsigned nb = blocks_for(a.n_cubes);
    hipLaunchKernelGGL(k_mesh_count, dim3(nb), dim3(DENSE_THREADS), 0, s, a, cfg, block_sums);
    hipLaunchKernelGGL(k_mesh_scan, dim3(1), dim3(1024), 0, s, block_sums, (int)nb, block_off, total);
}

void launch_mesh_emit(const DenseArgs& a, const uint8_t* cfg, const uint64_t* block_off, float* tris, float* cols,
                      int64_t cap, hipStream_t s) {
    hipLaunchKernelGGL(k_mesh_emit, dim3(blocks_for(a.n_cubes)), dim3(DENSE_THREADS), 0, s, a, cfg, block_off, tris, cols,
                       cap);
}

// one windowed pass along an axis of a volume [outer][n][ncol]-shaped by strides: x (stride 1,
// rows = every (y, z)), or y / z (columns = x, or x * y for z); LDS-staged for R <= EDT_LDS_R
static void edt_pass(const int32_t* in, int32_t* out, int64_t total, int nx, int64_t rows, int axis_n, int64_t stride,
                     int64_t plane, int ncol, int64_t planes, bool x_axis, int R, int32_t cap, hipStream_t s) {
    if (R > EDT_LDS_R) {
        hipLaunchKernelGGL(k_edt_pass, dim3(blocks_for(total)), dim3(DENSE_THREADS), 0, s, in, out, total, axis_n, stride,
                           R, cap);
    } else if (x_axis) {
        const int64_t tiles = (nx + DENSE_THREADS - 1) / DENSE_THREADS;
        hipLaunchKernelGGL(k_edt_pass_x_lds, dim3((unsigned)(rows * tiles)), dim3(DENSE_THREADS), 0, s, in, out, nx, rows,
                           R, cap);
    } else {
        const int64_t nblk = (int64_t)((ncol + 63) / 64) * ((axis_n + EDT_TA - 1) / EDT_TA) * planes;
        const size_t lds = sizeof(int32_t) * 64 * (EDT_TA + 2 * R);
        hipLaunchKernelGGL(k_edt_pass_yz_lds, dim3((unsigned)nblk), dim3(DENSE_THREADS), lds, s, in, out, ncol, axis_n,
                           stride, plane, R, cap);
    }
}

void launch_esdf(const DenseArgs& a, int R, const float* tab, int32_t* g0, int32_t* g1, float* out, hipStream_t s) {
    const int64_t nv = a.n_voxels, sy = a.nx, sz = (int64_t)a.nx * a.ny;
    const unsigned nb = blocks_for(nv);
    hipLaunchKernelGGL(k_esdf_sites, dim3(nb), dim3(DENSE_THREADS), 0, s, a, g0);
    edt_pass(g0, g1, nv, a.nx, (int64_t)a.ny * a.nz, a.nx, 1, 0, a.nx, 1, true, R, a.cap, s);              // x
    edt_pass(g1, g0, nv, a.nx, 0, a.ny, sy, sz, a.nx, a.nz, false, R, a.cap, s);                          // y: planes z
    edt_pass(g0, g1, nv, a.nx, 0, a.nz, sz, 0, (int)sz, 1, false, R, a.cap, s);                            // z: columns x*y
    hipLaunchKernelGGL(k_esdf_finish, dim3(nb), dim3(DENSE_THREADS), 0, s, a, g1, tab, out);
}

void launch_esdf_slice(const DenseArgs& a, int y0, int y1, int R, const float* tab, int32_t* g0, int32_t* g1,
                       uint8_t* obs, float* out, hipStream_t s) {
    const int64_t nc = (int64_t)a.nx * a.nz;
    const unsigned nb = blocks_for(nc);
    hipLaunchKernelGGL(k_esdf_slice_sites, dim3(nb), dim3(DENSE_THREADS), 0, s, a, y0, y1, g0, obs);
    edt_pass(g0, g1, nc, a.nx, a.nz, a.nx, 1, 0, a.nx, 1, true, R, a.cap, s);                              // x
    edt_pass(g1, g0, nc, a.nx, 0, a.nz, a.nx, 0, a.nx, 1, false, R, a.cap, s);                             // z
    hipLaunchKernelGGL(k_esdf_slice_finish, dim3(nb), dim3(DENSE_THREADS), 0, s, a, g0, obs, tab, out);
}
