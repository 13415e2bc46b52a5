"""Build guards (CPU) on the shipped gfx950 code: no cross-lane swap runs under a narrowed EXEC, and the
production fused kernels keep their scratch (VGPR-spill) footprint small.

The v4 kernels and the fused layer-wise form reduce across lanes with v_permlane16_swap /
v_permlane32_swap; a butterfly is only right when every lane takes part, and the compiler once sank
such swaps into EXEC-narrowed code (v5's bisect, profiles/r03/bisect_*.txt).  tools/exec_scan.py runs a
forward dataflow of the SI control-flow lowering's EXEC masks over every function of every code object
in libcet.so and reports each swap reached inside an open divergent region.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "channelestimationtransformer_amd", "libcet.so")

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                                reason="needs the ROCm llvm-objdump")


def test_no_lane_swap_under_narrowed_exec_in_libcet():
    import exec_scan

    if not os.path.exists(LIB):
        pytest.skip("libcet.so not built")
    findings, counted = exec_scan.scan(LIB)
    assert counted > 1000, f"only {counted} cross-lane swaps found: the scan did not see the v4 kernels"
    assert not findings, "\n".join(" ".join(f) for f in findings[:20])


def _fn(lines):
    """A synthetic function body in llvm-objdump's format (4-byte instructions from 0x100)."""
    out = ["0000000000000100 <f>:"]
    for i, ins in enumerate(lines):
        out.append(f"\t{ins:58s}// {0x100 + 4 * i:012X}: 00000000")
    return "\n".join(out)


@pytest.mark.parametrize("lines,flag", [
    # a swap inside an if-region: flagged
    (["v_cmp_gt_u32_e32 vcc, 16, v0", "s_and_saveexec_b64 s[4:5], vcc", "s_cbranch_execz 2",
      "v_permlane16_swap_b32_e32 v1, v2", "s_or_b64 exec, exec, s[4:5]", "s_endpgm"], True),
    # the same swap after the region is closed: clean
    (["v_cmp_gt_u32_e32 vcc, 16, v0", "s_and_saveexec_b64 s[4:5], vcc", "s_cbranch_execz 1",
      "v_mov_b32_e32 v3, v4", "s_or_b64 exec, exec, s[4:5]", "v_permlane16_swap_b32_e32 v1, v2",
      "s_endpgm"], False),
    # if / else: swap in the else arm flagged
    (["v_cmp_gt_u32_e32 vcc, 16, v0", "s_and_saveexec_b64 s[4:5], vcc", "s_xor_b64 s[4:5], exec, s[4:5]",
      "v_mov_b32_e32 v3, v4", "s_or_saveexec_b64 s[6:7], s[4:5]", "s_xor_b64 exec, exec, s[6:7]",
      "v_permlane32_swap_b32_e32 v1, v2", "s_or_b64 exec, exec, s[6:7]", "s_endpgm"], True),
    # a divergent loop: the swap after its exit is clean, one inside its body is flagged
    (["s_mov_b64 s[8:9], 0", "v_add_u32_e32 v0, 1, v0", "v_cmp_le_u32_e32 vcc, 5, v0",
      "s_or_b64 s[8:9], vcc, s[8:9]", "s_andn2_b64 exec, exec, s[8:9]", "s_cbranch_execnz 65531",
      "s_or_b64 exec, exec, s[8:9]", "v_permlane16_swap_b32_e32 v1, v2", "s_endpgm"], False),
    (["s_mov_b64 s[8:9], 0", "v_add_u32_e32 v0, 1, v0", "v_permlane16_swap_b32_e32 v1, v2",
      "v_cmp_le_u32_e32 vcc, 5, v0", "s_or_b64 s[8:9], vcc, s[8:9]", "s_andn2_b64 exec, exec, s[8:9]",
      "s_cbranch_execnz 65530", "s_or_b64 exec, exec, s[8:9]", "s_endpgm"], True),
])
def test_scan_flags_swaps_in_divergent_regions(lines, flag):
    import exec_scan

    (name, body), = list(exec_scan.functions(_fn(lines)))
    assert bool(exec_scan.scan_function(body)) == flag


# The production C2 instance's scratch per lane (tools/kernel_resources.py): 52 B since the once-per-call copy
# loops stopped hoisting their per-lane addresses (136 B before, which wrote 26 MiB of spill
# scratch per launch).  A regression past this budget brings the spill traffic back.
SCRATCH_BUDGET = {
    # the bf16 production instances (generic, C2, E43, encoder split; register-path decoder, bf16 decoder)
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi0ELb0ELi0ELb0ELb0ELi0E": 64,
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi0ELb0ELi1ELb0ELb0ELi0E": 64,    # C2 production (bf16)
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi0ELb0ELi2ELb0ELb0ELi0E": 64,
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi0ELb1E": 64,
    # the split-bf16 production instances: no private memory at all.  The round-4 ab8 reordering's wrong element
    # travelled with its address-taken K/V weight struct kept in private memory (320 B per lane here, 60 scratch
    # stores and 228 scratch loads), so a split-bf16 instance that grows a private segment is the
    # first thing to look at
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi1ELb0E": 0,
    "_ZN3cet2v419informer_forward_v4ILi128ELb0ELi1ELb0E": 0,
    # the mixed policy (bf16 encoder, split-bf16 decoder at the 128-VGPR cap: the decoder's hi/lo operands spill)
    "_ZN3cet2v419informer_forward_v4ILi64ELb0ELi0ELb0ELi1ELb0ELb0ELi1E": 400,
    "_ZN3cet2v422transformer_forward_v4ILi64ELb0E": 16,         # C3 production
    # fused layer-wise form, d_model <= 64: 16-24 B until round 5; 52 B (≤ 17 VGPRs) with the register attention
    # inlined at its three call sites, which runs a d_model-64, 4-head plan 17 % (fp32) / 25 % (bf16) faster
    # (profiles/r05/lw_generic/ab.log)
    "_ZN3cet2lw8lw_fusedILi4ELb0E": 64,
    "_ZN3cet2lw8lw_fusedILi4ELb1E": 128,                        # its compile-time d64-checkpoint layout
}


def test_production_kernels_scratch_budget():
    import kernel_resources

    if not os.path.exists(LIB):
        pytest.skip("libcet.so not built")
    res = kernel_resources.resources(LIB)
    for prefix, budget in SCRATCH_BUDGET.items():
        hits = {n: v for n, v in res.items() if n.startswith(prefix)}
        assert hits, f"kernel {prefix}… not found in libcet.so"
        for name, v in hits.items():
            assert v.get("private_segment_fixed_size", 0) <= budget, (name, v)
