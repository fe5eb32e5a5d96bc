"""Register-allocation guard for the shipped gfx950 kernels (CPU-only).

The temporal-blocking Jacobi kernel is VALU-issue bound at 2 waves per SIMD
with its allocation at 243-253 VGPRs; two unrelated one-line changes have
spilled it before (profiles/r02_tb.md 9.2/9.4), and a spill doubles the
pass time without changing a single result bit — no numerics test can see
it.  This test reads the AMDGPU code-object metadata of the built
``libgmt.so`` (``llvm-objdump --offloading`` extracts the gfx950 objects,
``llvm-readelf --notes`` prints each kernel's resource descriptor) and
fails if any kernel uses scratch (private segment) or spills VGPRs, or if
a temporal-blocking instantiation the planner can pick is missing (SGPR
spills go to VGPR lanes, not memory, and are allowed).  The exact-form
K = 20 kernel, which spilled 8 B per lane until round 5, fits as well now;
gmt_jacobi5tb_max_sweeps(1) stays 18 (its calibration never made K = 20
exact worthwhile).
"""
import os
import re
import shutil
import subprocess

import pytest

from native_util import ROOT

LLVM = "/opt/rocm/llvm/bin"
LIB = os.path.join(ROOT, "gpu_mpi_tests_amd", "_lib", "libgmt.so")
# every K gmt_jacobi5tb_supported() accepts (csrc/kernels/jacobi5tb.hip)
SUPPORTED_K = list(range(1, 11)) + [12, 14, 16, 18, 20]
MAX_EXACT_K = 18  # gmt_jacobi5tb_max_sweeps(1)


def _kernels(tmp_path):
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("no llvm-objdump in /opt/rocm/llvm/bin")
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (make lib / __graft_entry__.build())")
    lib = tmp_path / "libgmt.so"
    shutil.copy(LIB, lib)
    # extracts <lib>.<i>.<triple> files next to the input (so: in tmp_path)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", str(lib)], check=True,
                   capture_output=True, cwd=tmp_path)
    objs = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in libgmt.so"
    out = {}
    for o in objs:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(o)], check=True,
                               capture_output=True, text=True).stdout
        # one metadata map per kernel: split at each ".name:" of a kernel entry
        for block in re.split(r"\n\s+- \.", notes):
            m = re.search(r"\.name:\s+(\S+)", "." + block)
            if not m or not m.group(1).startswith("_Z"):
                continue
            vals = {}
            for key in ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count"):
                k = re.search(r"\." + key + r":\s+(\d+)", "." + block)
                vals[key] = int(k.group(1)) if k else 0
            out[m.group(1)] = vals
    return out


def test_no_kernel_uses_scratch_or_spills(tmp_path):
    ks = _kernels(tmp_path)
    assert len(ks) > 20, sorted(ks)
    bad = {n: v for n, v in ks.items() if v["private_segment_fixed_size"] or v["vgpr_spill_count"]}
    assert not bad, "kernels with scratch or spills:\n" + "\n".join(
        f"{subprocess.run(['c++filt', n], capture_output=True, text=True).stdout.strip()}: {v}"
        for n, v in sorted(bad.items()))


def test_every_plannable_k_is_built_and_fits(tmp_path):
    ks = _kernels(tmp_path)
    tb = {}
    for name, v in ks.items():
        m = re.match(r"_ZN3gmt2tb16jacobi5tb_kernelILi(\d+)ELb([01])ELb([01])E", name)
        if m:
            tb[(int(m.group(1)), m.group(2) == "1", m.group(3) == "1")] = v
    for k in SUPPORTED_K:
        for exact in (False, True):
            for edge in (False, True):
                v = tb.get((k, exact, edge))
                assert v is not None, f"jacobi5tb_kernel<{k},{exact},{edge}> missing"
                assert v["vgpr_count"] <= 256, (k, exact, edge, v)
                if exact and k > MAX_EXACT_K:
                    continue  # built for the kernel API, never planned (see the module docstring)
                # 2 waves per SIMD (amdgpu_waves_per_eu(2)) without scratch
                assert v["private_segment_fixed_size"] == 0 and v["vgpr_spill_count"] == 0, (k, exact, edge, v)
    assert max(k for k, _, _ in tb) == max(SUPPORTED_K), sorted(tb)
