"""The build's machine-code guard (thor-slam_amd/csrc/isa_guard.py, run by the Makefile before the
library is linked): no kernel spills VGPRs or uses scratch, and no MFMA puts its destination over a
source.  CPU only: hipcc cross-compiles the gfx950 code these tests inspect."""

from __future__ import annotations

import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "thor-slam_amd" / "csrc"
sys.path.insert(0, str(CSRC))
import isa_guard  # noqa: E402

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
needs_hipcc = pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not installed")

# 8 waves/SIMD leave 64 VGPRs; 96 values live across the loop do not fit, so the build spills
SPILL_SRC = r"""
#include <hip/hip_runtime.h>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
void k_forced_spill(const float* in, float* out, int n) {
    float v[96];
#pragma unroll
    for (int i = 0; i < 96; ++i) v[i] = in[threadIdx.x + 256 * i];
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 96; ++i) v[i] = v[i] * v[(i + 7) % 96] + v[(i + 31) % 96];
    }
#pragma unroll
    for (int i = 0; i < 96; ++i) out[threadIdx.x + 256 * i] = v[i];
}
// a private array read at a run-time index lives in scratch
__global__ void k_private_array(const int* idx, float* out) {
    float a[600];
    for (int i = 0; i < 600; ++i) a[i] = out[i * 64 + threadIdx.x];
    out[threadIdx.x] = a[idx[threadIdx.x] % 600];
}
"""


def _compile(src: Path, obj: Path, *extra: str) -> None:
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip", "-c", str(src), "-o", str(obj),
                    *extra], check=True, capture_output=True)


@needs_hipcc
def test_guard_passes_on_the_shipped_objects():
    objs = sorted((CSRC / "build").glob("*.o"))
    if not objs:
        pytest.skip("library not built (make -C thor-slam_amd/csrc)")
    assert isa_guard.check(objs) == []


@needs_hipcc
def test_guard_trips_on_a_forced_spill_build(tmp_path):
    src = tmp_path / "spill.hip"
    src.write_text(SPILL_SRC)
    obj = tmp_path / "spill.o"
    _compile(src, obj)
    errors = isa_guard.check([obj])
    assert any("k_forced_spill" in e and "spills" in e and "VGPRs" in e for e in errors), errors
    assert any("k_private_array" in e and "scratch" in e for e in errors), errors


@needs_hipcc
def test_guard_flags_mfma_destination_over_a_source(tmp_path):
    """tools/mfma_overlap_probe.hip pins the operand layouts in inline asm, including the spilling
    k_match build's two MFMAs; the guard must flag every overlapping layout and pass the disjoint
    reference and the exact accumulate (srcC == vdst)."""
    obj = tmp_path / "probe.o"
    _compile(ROOT / "tools" / "mfma_overlap_probe.hip", obj)
    errors = isa_guard.check([obj])
    flagged = {e.split(":")[1].strip() for e in errors}
    want = {"_Z6k_c_lo", "_Z6k_c_hi", "_Z6k_a_lo", "_Z6k_a_hi", "_Z6k_b_lo", "_Z6k_b_hi", "_Z8k_spill1", "_Z8k_spill2"}
    got = {f.split("P")[0] for f in flagged}
    assert want <= got, (want - got, errors)
    assert not any(("k_ref" in e) or ("k_mac" in e) for e in errors), errors
    spill1 = [e for e in errors if "k_spill1" in e][0]
    assert "srcA" in spill1 and "srcC (partial)" in spill1


# rule 3: in-launch hand-offs (k_ba_reduce_solve's pattern and three ways to break it)
HANDOFF_SRC = r"""
#include <hip/hip_runtime.h>
#define AGENT __HIP_MEMORY_SCOPE_AGENT
__device__ void tail(const double* C, double* out, int last) {
    if (!last) return;
    out[threadIdx.x] = __hip_atomic_load(C + threadIdx.x, __ATOMIC_RELAXED, AGENT) +
                       __hip_atomic_load(C + 256 + threadIdx.x, __ATOMIC_RELAXED, AGENT);
}
__global__ void k_handoff_ok(double* C, int* done, double* out, double v) {
    __shared__ int s_last;
    __hip_atomic_store(C + blockIdx.x * 256 + threadIdx.x, v, __ATOMIC_RELAXED, AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    tail(C, out, s_last);
}
__global__ void k_handoff_plain_store(double* C, int* done, double* out, double v) {
    __shared__ int s_last;
    C[blockIdx.x * 256 + threadIdx.x] = v;   // cached in this XCD's L2: the last block may not see it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    tail(C, out, s_last);
}
__global__ void k_handoff_no_wait(double* C, int* done, double* out, double v) {
    __shared__ int s_last;
    __hip_atomic_store(C + blockIdx.x * 256 + threadIdx.x, v, __ATOMIC_RELAXED, AGENT);
    if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    tail(C, out, s_last);
}
__global__ void k_handoff_plain_load(double* C, int* done, double* out, double v) {
    __shared__ int s_last;
    __hip_atomic_store(C + blockIdx.x * 256 + threadIdx.x, v, __ATOMIC_RELAXED, AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    if (s_last) out[threadIdx.x] = C[threadIdx.x] + C[256 + threadIdx.x];
}
"""


@needs_hipcc
def test_guard_checks_the_in_launch_handoff(tmp_path):
    """Rule 3 (the BA hand-off): published stores with sc1, drained before the
    counter, and sc1 loads in the last block.  The shipped k_ba_reduce_solve passes (the first
    test); each broken variant trips."""
    src = tmp_path / "handoff.hip"
    src.write_text(HANDOFF_SRC)
    obj = tmp_path / "handoff.o"
    _compile(src, obj)
    names = ("k_handoff_ok", "k_handoff_plain_store", "k_handoff_no_wait", "k_handoff_plain_load")
    errors = isa_guard.check([obj], handoff={n: 2 for n in names})
    by = {n: [e for e in errors if f"{n}" in e] for n in names}
    assert by["k_handoff_ok"] == [], errors
    assert any("without sc1" in e for e in by["k_handoff_plain_store"]), errors
    assert any("vmcnt(0)" in e for e in by["k_handoff_no_wait"]), errors
    assert any("sc1 (agent-scope) loads" in e for e in by["k_handoff_plain_load"]), errors
    # the library's own hand-off kernel is checked by default and must exist in k_ba's object
    objs = sorted((CSRC / "build").glob("*.o"))
    if objs:
        assert isa_guard.check([o for o in objs if o.name == "k_ba.hip.o"]) == []
