"""Register allocation of the configs[1] sparse-coding kernel, read from the built library (CPU).

k_ista_ln2 (the bb = 8 kernel, main_LRS_PnP.py:131-149) fills all 512 registers of its SIMD.  LLVM
gives the product instantiation <256, false, 1, true, 1> round 1's allocation (30-32 AGPRs, no
spills) only while ista.hip also instantiates <..., 0> (compiled alone the same source
keeps fewer allocas to the backend, ends at 82 AGPRs with 241 v_accvgpr moves, and configs[1] loses
2.8 %).  No source attribute controls it (amdgpu_waves_per_eu, amdgpu_num_vgpr and
amdgpu_flat_work_group_size all leave 82), so this test pins the result instead: a compiler update or
a change elsewhere in ista.hip that brings the 82-AGPR code back fails here, on the CPU, every round.
"""
import os
import re
import struct
import subprocess
import tempfile

import pytest

yaml = pytest.importorskip("yaml")   # PyYAML reads the code-object notes

from lrspnp import _lib

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PRODUCT = "_ZN3lrs10k_ista_ln2ILi256ELb0ELi1ELb1ELi1EEEvNS_10IstaParamsE"


def code_objects(so):
    """The gfx950 code objects (bytes) of `so`'s .hip_fatbin clang offload bundles."""
    sec = subprocess.run([READELF, "-S", "-W", so], capture_output=True, text=True, check=True).stdout
    m = re.search(r"\.hip_fatbin\s+PROGBITS\s+[0-9a-f]+\s+([0-9a-f]+)\s+([0-9a-f]+)", sec)
    assert m, "no .hip_fatbin section"
    off, size = int(m.group(1), 16), int(m.group(2), 16)
    with open(so, "rb") as f:
        f.seek(off)
        data = f.read(size)
    magic, out, pos = b"__CLANG_OFFLOAD_BUNDLE__", [], 0
    while (i := data.find(magic, pos)) >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                out.append(data[i + eo:i + eo + es])
        pos = i + 1
    return out


def _with_file(co, argv):
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as t:
        t.write(co)
    try:
        return subprocess.run(argv + [t.name], capture_output=True, text=True, check=True).stdout
    finally:
        os.unlink(t.name)


def kernel_metadata(so):
    """{kernel name: its amdhsa.kernels metadata} of every gfx950 code object in `so`'s fat binary."""
    out = {}
    for co in code_objects(so):
        notes = _with_file(co, [READELF, "--notes"])
        doc = notes[notes.index("---"):]
        doc = doc[:doc.index("\n...")] if "\n..." in doc else doc
        for k in yaml.safe_load(doc).get("amdhsa.kernels", []):
            out[k[".name"]] = k
    return out


def mfma_loops(so):
    """{kernel symbol: [(MFMAs, conditional branches, s_waitcnt vmcnt(0)) per loop that issues MFMAs]}:
    a loop = the instructions from a backward branch's target to the branch (llvm-objdump)."""
    res = {}
    for co in code_objects(so):
        txt = _with_file(co, [OBJDUMP, "-d", "--mcpu=gfx950"])
        starts, body, cur = {}, {}, None
        for line in txt.splitlines():
            m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
            if m:
                cur = m.group(2)
                starts[cur] = int(m.group(1), 16)
                body[cur] = []
                continue
            m = re.search(r"//\s*([0-9A-F]+):", line)
            if cur and m:
                body[cur].append((int(m.group(1), 16), line.strip()))
        for name, ins in body.items():
            loops = []
            for k, (a, x) in enumerate(ins):
                m = re.search(r"s_(?:cbranch_\w+|branch)\s.*<(\S+)\+0x([0-9a-f]+)>", x)
                if not m or m.group(1) not in starts:
                    continue
                tgt = starts[m.group(1)] + int(m.group(2), 16)
                if tgt >= a:
                    continue
                seg = [y for b, y in ins[:k] if b >= tgt]
                nm = sum("v_mfma" in y for y in seg)
                if nm:
                    loops.append((nm, sum("s_cbranch" in y for y in seg), sum("s_waitcnt vmcnt(0)" in y for y in seg)))
            if loops:
                res[name] = loops
    return res


@pytest.fixture(scope="module")
def meta():
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not found")
    return kernel_metadata(_lib.LIB_PATH)


def test_ista_ln2_register_allocation(meta):
    k = meta.get(PRODUCT)
    assert k is not None, "the product k_ista_ln2 instantiation is missing from the library"
    assert k[".agpr_count"] <= 32, f"k_ista_ln2 AGPRs {k['.agpr_count']} > 32: round 1's allocation is lost"
    assert k[".vgpr_count"] <= 288 and k[".vgpr_spill_count"] == 0 and k[".private_segment_fixed_size"] == 0


# kernels allowed scratch: the eigensolver's per-thread arrays (by design, one workgroup off the
# critical path), the f32-product ISTA option and the single-row-tile k_ista_rs form (never on a
# benched path), and the 196^2 register BatchNorm backward k_bn_bwd_r<10> (8 registers of its 80
# register-held values at 1024 threads: 36 B per lane that stay in L1/L2, less traffic than
# re-reading z for x_hat, 19.7 MB per layer)
SCRATCH_OK = ("k_svt_eig", "k_jacobi", "k_ista_res", "k_ista_rsILi16ELi2ELi1E", "k_bn_bwd_rILi10E")


def test_no_scratch_in_hot_kernels(meta):
    """No benched-path kernel spills to scratch (a spill costs many times its bytes in fabric
    traffic: DESIGN §4, the 128-register k_ista_pat variant)."""
    bad = [(n, k[".private_segment_fixed_size"]) for n, k in meta.items()
           if k[".private_segment_fixed_size"] > 0 and not any(h in n for h in SCRATCH_OK)]
    assert not bad, bad


# The implicit-GEMM conv loops after round 5's branch-free loaders: a loader that wrote
# "c < Cin ? load : 0" per channel put ~16 conditional branches into every k-loop and, with them, a
# drain of every load in flight (s_waitcnt vmcnt(0)) at the loop head, which cost the 196^2 step
# 20 us and the 36^2 step 13 us.  Bounds per MFMA loop: (conditional branches, vmcnt(0) waits).
LOOP_BOUNDS = {
    "_ZN3lrs9k_gemm_s3INS_5LdPreENS_7LdFwdTMEEEvNS_8GemmArgsET_T0_": (2, 1),
    "_ZN3lrs9k_gemm_s3INS_5LdPreENS_9LdDgradTMEEEvNS_8GemmArgsET_T0_": (2, 1),
    "_ZN3lrs9k_gemm_s3INS_5LdPreENS_9LdUpFwdTMEEEvNS_8GemmArgsET_T0_": (2, 1),
    "_ZN3lrs9k_gemm_s3INS_5LdPreENS_11LdUpDgradTMEEEvNS_8GemmArgsET_T0_": (2, 1),
    "_ZN3lrs9k_conv_smINS_5SmFwdENS_5SmPreEEEvNS_8GemmArgsET0_T_": (4, 1),
    "_ZN3lrs9k_conv_smINS_5SmAdjENS_5SmPreEEEvNS_8GemmArgsET0_T_": (10, 3),
    "_ZN3lrs9k_conv_smINS_7SmWgradENS_7SmDenseEEEvNS_8GemmArgsET0_T_": (2, 1),
}


def test_conv_loops_keep_their_loads_in_flight():
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not found")
    loops = mfma_loops(_lib.LIB_PATH)
    for name, (br, vm) in LOOP_BOUNDS.items():
        assert name in loops, f"{name}: no MFMA loop found"
        for nm, nb, nv in loops[name]:
            assert nb <= br and nv <= vm, (name, nm, nb, nv)
