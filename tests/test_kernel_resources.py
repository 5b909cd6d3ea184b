"""Build-time guard: the hot kernels of the built libp3d.so use NO scratch.

A private array indexed with a value the compiler cannot resolve to a constant after unrolling is
placed in scratch memory (AMDGPU promotes an array to registers only when every index is constant),
and so is a register spill.  Either way its private_segment_fixed_size becomes non-zero.  The
persistent kernels sit at the register limit with runtime-bounded loops over private arrays
(k_gemv_chain's wf / acc / e, k_serve6's rings); a runtime index that can leave its array is only
possible once the array lives in scratch, and the round-4 chain build that spilled faulted on its
first box run.  This test reads the gfx950 code object's metadata in the build
container (tools/kernel_resources.py: no GPU), so a future spill fails here, not on the box.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "3d-pose-baseline_amd", "libp3d.so")

# the kernels on the default paths (rocprof names); every one must be spill- and scratch-free
HOT = [
    "void k_gemv_chain<4, 4>(GemvChain)",            # batch <= 4 forward, one launch
    "void k_serve6<4, 3, 2, 5, true>(ServeArgs)",     # the headline: 20 batch-64 requests per launch (pair form)
    "void k_serve6<4, 3, 2, 10, false>(ServeArgs)",   # the same rows as one 160-row unit per XCD (P3D_SERVE6_PAIR=0)
    "void k_serve6<4, 3, 2, 1, false>(ServeArgs)",           # one batch-64 request
    "void k_serve6<4, 3, 2, 2, false>(ServeArgs)",
    "void k_gemm_bf16p<64, 4, 8, false, 0, false>",   # cfg5 hidden layer
    "k_wgrad_multi",                      # cfg3 weight gradients + fused TF1 Adam
    "k_adam_pack",                                    # DP optimizer
    "void k_fwd<1, 8, 8, 2, true, true, 1>(FwdArgs)",  # BN-train hidden forward (exchange form)
    "void k_dgrad<1, 16, 4, 2, true, 1>",             # hidden data gradient (16 waves, default)
    "void k_fwd<1, 16, 4, 2, true, false, 2>",        # inference output layer (16 waves split K)
    "void k_fwd<1, 16, 4, 2, true, true, 1>",
    "void k_gemm_f32<2, 2, true>",                    # cfg4 large-M hidden layer
    "void k_gemm_f32<2, 2, false>",                   # cfg4 large-M input layer
]


def _resources():
    if not os.path.exists(LIB):
        pytest.skip("libp3d.so not built")
    if not all(os.path.exists(os.path.join("/opt/rocm/lib/llvm/bin", t))
               for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")):
        pytest.skip("ROCm LLVM tools not present")
    from tools.kernel_resources import kernel_resources
    return kernel_resources(LIB)


@pytest.fixture(scope="module")
def res():
    return _resources()


def _find(res, name):
    if name in res:
        return res[name]
    # match on the kernel and its template arguments (the argument list left out)
    head = name.split("(")[0]
    hits = [k for k in res if k.split("(")[0] == head]
    assert hits, "kernel %s not in the code object (renamed? update HOT)" % name
    return res[hits[0]]


@pytest.mark.parametrize("name", HOT)
def test_hot_kernel_uses_no_scratch(res, name):
    r = _find(res, name)
    assert r.get("private_segment_fixed_size", 0) == 0, (name, r)
    # (SGPR spills go to VGPR lanes, v_writelane / v_readlane: no memory.)  VGPR spills: none, except
    # into the accumulation registers -- the pair form's prologue spills 2 VGPRs while it holds unit
    # B's input operands across unit A's post (round 6); with no scratch segment those can only be
    # AGPR copies (v_accvgpr_write / read), never memory
    spills = r.get("vgpr_spill_count", 0)
    assert spills == 0 or (name.startswith("void k_serve6<4, 3, 2, 5, true>") and spills <= 2), (name, r)
    assert not r.get("uses_dynamic_stack", False), (name, r)


def test_no_kernel_uses_dynamic_stack(res):
    """No kernel calls a function with a run-time stack (an un-inlined call: its stack size is a
    runtime default, not something the metadata bounds)."""
    bad = [k for k, r in res.items() if r.get("uses_dynamic_stack")]
    assert not bad, bad


@pytest.mark.parametrize("name", ["k_wgrad_multi", "k_wgrad_grad"])
def test_weight_gradient_kernels_fit_four_per_cu(res, name):
    """1,024 of cfg3's 1,056 weight-gradient tiles in the first round needs four 256-thread
    workgroups per CU: <= 40 KB of LDS (4 x 40 KB = the CU's 160 KB) and <= 128 registers (VGPR +
    AGPR: 4 waves per SIMD).  (Round 4's 41 KB / 131-register form held three: 768 + 288 tiles.)"""
    r = _find(res, name)
    assert r.get("group_segment_fixed_size", 0) <= 40960, (name, r)
    assert r.get("vgpr_count", 0) + r.get("agpr_count", 0) <= 128, (name, r)


def test_pair_form_post_wait_follows_its_refills():
    """k_serve6's pair form posts a block's flag after `s_waitcnt vmcnt(DEPTH (RT +
    NCM))` -- the previous block's epilogue stores are acknowledged once no more than the round's
    refill loads are outstanding, which holds only while at least that many vector-memory operations
    follow the stores in the emitted code (vmcnt retires in issue order).  A compiler change that
    hoisted a refill above the stores, or dropped one, would let the flag overtake the stores:
    silent stale reads.  The wait is marked (`s_nop 5`, p3d_serve6.h); walking back from every
    marked wait to the nearest store or label must cross at least DEPTH (RT + NCM) = 4 (5 + 2) = 28
    vector loads (a label ends the count early, so the count is a lower bound: a conservative
    check)."""
    import re
    if not os.path.exists(LIB):
        pytest.skip("libp3d.so not built")
    from tools.kernel_resources import kernel_isa
    isa = kernel_isa("void k_serve6<4, 3, 2, 5, true>", LIB)
    need = 4 * (5 + 2)
    marks = [i for i in range(len(isa) - 1)
             if "s_waitcnt vmcnt(%d)" % need in isa[i] and "s_nop 5" in isa[i + 1]]
    assert marks, "the marked post wait is missing from the pair kernel"
    vmem = re.compile(r"\s(buffer|global|flat|scratch)_(\w+)")
    label = re.compile(r"^[0-9a-f]{16} <")
    for i in marks:
        loads, j = 0, i - 1
        while j > 0 and not label.match(isa[j]):
            m = vmem.search(isa[j])
            if m and ("store" in m.group(2) or "atomic" in m.group(2)):
                break
            if m:
                loads += 1
            j -= 1
        assert loads >= need, (i, loads, isa[j].strip())
