"""The in-flight scalar-load check (tools/check_smem_inflight.py) on the shipped gfx950
code, and on hand-made instruction sequences that must and must not be flagged (among them the round-2
fault's pattern: child offsets loaded into prefetch sinks that a late load then overwrote)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_smem_inflight as C  # noqa: E402

LIB = os.path.join(ROOT, "ray-tracing-project_amd", "lib", "librtamd.so")


def run(seq):
    """Instructions as (mnemonic, operands[, branch target index]) -> findings."""
    ins = []
    for k, x in enumerate(seq):
        tgt = 4 * x[2] if len(x) > 2 else None
        ins.append((4 * k, x[0], x[1], tgt))
    return C.check_function("f", ins, calls_wait=True)


def test_flags_write_of_inflight_destination():
    f = run([("s_load_dword", "s10, s[0:1], 0x0"), ("s_mov_b32", "s10, 0"), ("s_waitcnt", "lgkmcnt(0)"),
             ("s_endpgm", "")])
    assert len(f) == 1 and "writes s10" in f[0]


def test_flags_read_of_inflight_destination():
    f = run([("s_load_dwordx2", "s[10:11], s[0:1], 0x0"), ("s_add_u32", "s12, s11, 1"), ("s_endpgm", "")])
    assert len(f) == 1 and "reads s11" in f[0]


def test_partial_wait_does_not_retire_scalar_loads():
    f = run([("s_load_dword", "s10, s[0:1], 0x0"), ("s_waitcnt", "lgkmcnt(1)"), ("v_mov_b32_e32", "v0, s10"),
             ("s_endpgm", "")])
    assert len(f) == 1


def test_wait_retires_and_loop_carried_sink_is_clean():
    # the carried-prefetch form: the loop's own node load waits, then prefetches into a sink that is only
    # ever loaded again (never read or written) until the next wait
    seq = [("s_mov_b32", "s20, 0"),                            # 0
           ("s_load_dwordx16", "s[0:15], s[30:31], s20"),      # 1 loop head: node load
           ("s_waitcnt", "lgkmcnt(0)"),                        # 2
           ("s_load_dword", "s40, s[30:31], s14"),             # 3 prefetch child 0 into the sink
           ("s_load_dword", "s40, s[30:31], s15"),             # 4 prefetch child 1 into the same sink
           ("s_mov_b32", "s20, s12"),                          # 5 next node
           ("s_cmp_lg_u32", "s20, 0"),                         # 6
           ("s_cbranch_scc1", "", 1),                          # 7 back to the node load (its wait retires)
           ("s_waitcnt", "lgkmcnt(0)"),                        # 8
           ("s_endpgm", "")]
    assert run(seq) == []


def test_flags_round2_fault_pattern():
    # offsets loaded into the sink registers while the previous step's prefetch into them is in flight,
    # then used as the next prefetch's offset: either load may have written the register last
    seq = [("s_load_dword", "s40, s[30:31], s14"),             # previous step's prefetch (sink s40)
           ("s_load_dwordx16", "s[0:15], s[30:31], s20"),
           ("s_load_dword", "s40, s[30:31], s20 offset:0x38"), # child offset into the same register
           ("s_waitcnt", "lgkmcnt(0)"),
           ("s_load_dword", "s41, s[30:31], s40"),             # prefetch at that offset
           ("s_waitcnt", "lgkmcnt(0)"),
           ("s_endpgm", "")]
    f = run(seq)
    assert len(f) == 1 and "raced" in f[0]


def test_long_branch_is_followed():
    # s_getpc / s_add / s_addc / s_setpc to index 7, where the in-flight destination is read
    seq = [("s_load_dword", "s10, s[0:1], 0x0"),               # 0 @0
           ("s_getpc_b64", "s[2:3]"),                          # 1 @4 (pc = 8)
           ("s_add_u32", "s2, s2, 0x14"),                      # 2 @8  -> 8 + 0x14 = 0x1c = index 7
           ("s_addc_u32", "s3, s3, 0"),                        # 3
           ("s_setpc_b64", "s[2:3]"),                          # 4
           ("s_waitcnt", "lgkmcnt(0)"),                        # 5 (skipped by the branch)
           ("s_endpgm", ""),                                   # 6
           ("v_mov_b32_e32", "v0, s10"),                       # 7
           ("s_endpgm", "")]
    f = run(seq)
    assert len(f) == 1 and "reads s10" in f[0]


@pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which("objcopy") or
                    not os.path.exists(os.path.join(C.LLVM, "llvm-objdump")), reason="library or ROCm tools missing")
def test_shipped_library_has_no_inflight_hazard():
    checked, problems = C.check_library(LIB)
    assert checked > 20, checked
    assert problems == [], "\n".join(problems[:20])


def run_v(seq):
    ins = []
    for k, x in enumerate(seq):
        tgt = 4 * x[2] if len(x) > 2 else None
        ins.append((4 * k, x[0], x[1], tgt))
    return C.check_vmem("f", ins, C.cfg("f", ins), calls_wait=True)


def test_vector_loads_in_order_retirement():
    # two loads, vmcnt(1): the first has landed, the second may not have
    base = [("global_load_dword", "v5, v0, s[2:3]"), ("global_load_dword", "v6, v1, s[2:3]"),
            ("s_waitcnt", "vmcnt(1)")]
    assert run_v(base + [("v_add_f32_e32", "v7, v5, v5"), ("s_endpgm", "")]) == []
    f = run_v(base + [("v_add_f32_e32", "v7, v6, v6"), ("s_endpgm", "")])
    assert len(f) == 1 and "v6" in f[0]
    # a carried prefetch sink reloaded every iteration and retired only after the loop is clean
    loop = [("v_mov_b32_e32", "v9, 0"), ("global_load_dword", "v9, v0, s[2:3]"), ("s_cmp_lg_u32", "s4, 0"),
            ("s_cbranch_scc1", "", 1), ("s_waitcnt", "vmcnt(0)"), ("v_mov_b32_e32", "v9, 1"), ("s_endpgm", "")]
    assert run_v(loop) == []
    # ... but not if the loop body copies it
    bad = loop[:2] + [("v_mov_b32_e32", "v10, v9")] + loop[2:]
    bad[4] = ("s_cbranch_scc1", "", 1)
    assert len(run_v(bad)) == 1
