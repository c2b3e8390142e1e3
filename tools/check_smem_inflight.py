#!/usr/bin/env python3
"""Static check of the library's gfx950 code for in-flight scalar loads.

The traversal loops issue scalar loads from inline asm whose completion the compiler does not track:
prefetches into "sink" SGPRs, carried across loop iterations and retired by a later s_waitcnt (node
loads, child prefetches: rt_device.hip sload_node_pf_carry, traverse_wide_fast). Scalar loads return
out of order and write their destination whenever the data arrives, so between such a load and the next
`s_waitcnt lgkmcnt(0)` no instruction may read its destination SGPRs (stale value), write them (the late
load would overwrite the new value: the round-2 fault, profiles/ab/r02_pf_carry_ab.txt), or copy them.
Two loads in flight into the same SGPR (the prefetch sink) are allowed, but after the wait that register
holds either value, so it must not be read before something else writes it.

The check runs on what the GPU executes: the gfx950 code objects bundled in librtamd.so, disassembled
with the ROCm llvm-objdump, one control-flow graph per function (branch targets from the disassembly), and
a forward data-flow fixpoint over the set of in-flight destination SGPRs (joined by union at merges:
an SGPR pending on any path into an instruction counts as pending there). A call (s_swappc) with a scalar
load in flight is also an error. Exit status 1 and one line per finding when anything is violated.

Usage: check_smem_inflight.py [librtamd.so] [--function SUBSTRING]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def disassemble(lib):
    """Disassembly text of every gfx950 code object bundled in the shared library's .hip_fatbin."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        sec = os.path.join(td, "fatbin.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, sec], check=True)
        data = open(sec, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            b = os.path.join(td, f"b{i}.bin")
            co = os.path.join(td, f"b{i}.co")
            open(b, "wb").write(data[s:e])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            d = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                               check=True)
            out.append(d.stdout)
    return "\n".join(out)


FUNC_RE = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
INS_RE = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):")
TARGET_RE = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>|<([^>+]+)>")
SREG_RE = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def parse_functions(text):
    """{name: [(addr, mnemonic, operand text), ...]} in address order."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = FUNC_RE.match(line)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            base = int(m.group(1), 16)
            continue
        if cur is None:
            continue
        m = INS_RE.match(line)
        if not m:
            continue
        mnem, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if mnem.startswith("s_branch") or mnem.startswith("s_cbranch"):
            t = TARGET_RE.search(line.split("//", 1)[1])
            if t:
                tgt = base + (int(t.group(2), 16) if t.group(2) else 0)
        cur.append((addr, mnem, ops.split("//")[0].strip(), tgt))
    return funcs


def sregs(tok_text):
    """SGPR numbers named in an operand string (vcc / exec / ttmp / m0 are never load destinations here)."""
    regs = []
    for m in SREG_RE.finditer(tok_text):
        if m.group(3) is not None:
            regs.append(int(m.group(3)))
        else:
            regs.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


NO_DST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_endpgm", "s_setpc", "s_sleep",
          "s_barrier", "s_setprio", "s_sendmsg", "s_trap", "s_icache", "s_ttrace", "ds_", "global_store",
          "buffer_store", "flat_store", "scratch_store", "v_writelane", "s_set_gpr_idx")
SECOND_DST = ("v_add_co_", "v_sub_co_", "v_subrev_co_", "v_addc_co_", "v_subb_co_", "v_subbrev_co_", "v_div_scale",
              "v_mad_u64_u32", "v_mad_i64_i32")


def classify(mnem, ops):
    """(read SGPRs, written SGPRs) of one instruction, from its explicit operands."""
    parts = [p.strip() for p in ops.split(",")] if ops else []
    if not parts:
        return [], []
    if mnem.startswith(NO_DST):
        return sregs(ops), []
    if mnem.startswith(SECOND_DST) and len(parts) > 1:
        w = sregs(parts[1])
        r = sregs(",".join(parts[2:]))
        return r, w
    # SALU / SMEM / VALU with an SGPR destination (v_cmp_*_e64, v_readlane, v_readfirstlane): first operand
    w = sregs(parts[0])
    r = sregs(",".join(parts[1:]))
    return r, w


def is_smem_load(mnem):
    return mnem.startswith(("s_load_", "s_buffer_load_", "s_scratch_load_"))


def lgkm_zero(mnem, ops):
    return mnem == "s_waitcnt" and ("lgkmcnt(0)" in ops or ops.strip() in ("0", "0x0"))


def is_return(ops):
    return ops.replace(" ", "") == "s[30:31]"


def _imm(x):
    x = x.strip()
    v = int(x, 16) if x.lower().startswith(("0x", "-0x")) else int(x)
    return v & 0xFFFFFFFF


def long_branch_target(ins, i):
    """Target of a long branch: s_getpc_b64 s[a:b]; s_add_u32 sa, sa, lo; s_addc_u32 sb, sb, hi; s_setpc_b64."""
    regs = ins[i][2].replace(" ", "")
    lo = hi = pc = None
    for j in range(i - 1, max(i - 8, -1), -1):
        _, m, ops, _ = ins[j]
        p = [x.strip() for x in ops.split(",")]
        if m == "s_addc_u32" and hi is None and len(p) == 3:
            hi = _imm(p[2])
        elif m == "s_add_u32" and lo is None and len(p) == 3:
            lo = _imm(p[2])
        elif m == "s_getpc_b64" and ops.replace(" ", "") == regs:
            pc = ins[j + 1][0]
            break
    if lo is None or hi is None or pc is None:
        return None
    off = (hi << 32) | lo
    if off >= 1 << 63:
        off -= 1 << 64
    return pc + off


VREG_RE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("global_", "buffer_", "scratch_", "flat_")


def vregs(text):
    regs = []
    for m in VREG_RE.finditer(text):
        if m.group(3) is not None:
            regs.append(int(m.group(3)))
        else:
            regs.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


def vmcnt_of(mnem, ops):
    """The vmcnt threshold of an s_waitcnt (None: does not wait on vector memory)."""
    if mnem != "s_waitcnt":
        return None
    if ops.strip() in ("0", "0x0"):
        return 0
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def cfg(name, ins):
    """Successor lists of a function's instructions (branch targets resolved, long branches followed)."""
    addr_idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    n = len(ins)
    succ = []
    for i, (a, mnem, ops, tgt) in enumerate(ins):
        s = []
        if mnem.startswith("s_setpc") and not is_return(ops):
            t = long_branch_target(ins, i)
            if t is None or t not in addr_idx:
                raise ValueError(f"{name} @{a:#x}: unresolved s_setpc target")
            s.append(addr_idx[t])
        elif mnem.startswith(("s_endpgm", "s_setpc")):
            pass
        elif mnem.startswith("s_branch"):
            if tgt in addr_idx:
                s.append(addr_idx[tgt])
        else:
            if i + 1 < n:
                s.append(i + 1)
            if mnem.startswith("s_cbranch") and tgt in addr_idx:
                s.append(addr_idx[tgt])
        succ.append(s)
    return succ


def check_vmem(name, ins, succ, calls_wait=False):
    """The same check for vector-memory loads into VGPRs (the asm prefetch sinks of RT_WIDE_PF 5 / 6 and
    everything the compiler emits). Vector loads return in issue order, so s_waitcnt vmcnt(N) retires
    every load with at least N vector-memory instructions issued after it; the state per pending VGPR is
    that count (the minimum over the paths reaching an instruction)."""
    n = len(ins)
    IN = [None] * n
    IN[0] = {}
    work = [0]
    findings = {}
    while work:
        i = work.pop()
        pend = dict(IN[i])
        a, mnem, ops, _ = ins[i]
        wn = vmcnt_of(mnem, ops)
        if wn is not None:
            pend = {x: v for x, v in pend.items() if v[0] < wn}
        elif mnem.startswith(VMEM):
            regs = vregs(ops)
            is_load = "_load" in mnem or ("_atomic" in mnem and " glc" in " " + ops)
            dst = set(vregs(ops.split(",")[0])) if is_load else set()
            for x in regs:
                if x in pend and x not in dst:
                    findings[(a, x)] = (f"{name} @{a:#x}: {mnem} {ops}: uses v{x} while a vector load into it is in "
                                        f"flight (load at {pend[x][1]:#x})")
            pend = {x: (min(64, c + 1), o) for x, (c, o) in pend.items()}
            for x in dst:
                pend[x] = (0, a)
        else:
            for x in vregs(ops):
                if x in pend:
                    findings[(a, x)] = (f"{name} @{a:#x}: {mnem} {ops}: touches v{x} while a vector load into it is "
                                        f"in flight (load at {pend[x][1]:#x})")
            if mnem.startswith("s_swappc") and calls_wait:
                pend = {}
        for j in succ[i]:
            if IN[j] is None:
                IN[j] = pend
                work.append(j)
                continue
            merged = dict(IN[j])
            for x, v in pend.items():
                if x not in merged or v[0] < merged[x][0]:
                    merged[x] = v
            if merged != IN[j]:
                IN[j] = merged
                work.append(j)
    return sorted(findings.values())


def check_function(name, ins, calls_wait=False):
    addr_idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    n = len(ins)
    succ = []
    for i, (a, mnem, ops, tgt) in enumerate(ins):
        s = []
        if mnem.startswith("s_setpc") and not is_return(ops):
            t = long_branch_target(ins, i)
            if t is None or t not in addr_idx:
                raise ValueError(f"{name} @{a:#x}: unresolved s_setpc target")
            s.append(addr_idx[t])
        elif mnem.startswith(("s_endpgm", "s_setpc")):
            pass
        elif mnem.startswith("s_branch"):
            if tgt in addr_idx:
                s.append(addr_idx[tgt])
        else:
            if i + 1 < n:
                s.append(i + 1)
            if mnem.startswith("s_cbranch") and tgt in addr_idx:
                s.append(addr_idx[tgt])
        succ.append(s)
    # state at entry of each instruction: (pending: {reg: 1 | 2}, ambiguous: frozenset)
    IN = [None] * n
    IN[0] = ({}, frozenset())
    work = [0]
    findings = {}

    def join(a, b):
        if a is None:
            return b
        p = dict(a[0])
        for k, v in b[0].items():
            c0, o0 = p.get(k, (0, frozenset()))
            p[k] = (max(c0, v[0]), o0 | v[1])
        return (p, a[1] | b[1])

    def origin(pend, x):
        return ", ".join(f"{o:#x}" for o in sorted(pend[x][1])[:4])

    while work:
        i = work.pop()
        pend, amb = IN[i]
        pend = dict(pend)
        amb = set(amb)
        a, mnem, ops, _ = ins[i]
        r, w = classify(mnem, ops)
        if is_smem_load(mnem):
            for x in r:
                if x in pend:
                    findings[(a, x)] = (f"{name} @{a:#x}: {mnem} {ops}: reads s{x} while a scalar load into it is in "
                                        f"flight (load at {origin(pend, x)})")
                elif x in amb:
                    findings[(a, x)] = f"{name} @{a:#x}: {mnem} {ops}: reads s{x}, which two loads raced to write"
            for x in w:
                c0, o0 = pend.get(x, (0, frozenset()))
                pend[x] = (min(2, c0 + 1), o0 | {a})
                amb.discard(x)
        elif lgkm_zero(mnem, ops):
            amb |= {x for x, (c, _) in pend.items() if c >= 2}
            pend = {}
        else:
            if mnem.startswith("s_swappc") and pend and not calls_wait:
                findings[(a, -1)] = (f"{name} @{a:#x}: call with scalar loads in flight into "
                                     + ", ".join(f"s{x} (load at {origin(pend, x)})" for x in sorted(pend)))
            for x in r:
                if x in pend:
                    findings[(a, x)] = (f"{name} @{a:#x}: {mnem} {ops}: reads s{x} while a scalar load into it is in "
                                        f"flight (load at {origin(pend, x)})")
                elif x in amb:
                    findings[(a, x)] = f"{name} @{a:#x}: {mnem} {ops}: reads s{x}, which two loads raced to write"
            for x in w:
                if x in pend:
                    findings[(a, x)] = (f"{name} @{a:#x}: {mnem} {ops}: writes s{x} while a scalar load into it is in "
                                        f"flight (load at {origin(pend, x)}; it may land later and overwrite it)")
                amb.discard(x)
            if mnem.startswith("s_swappc") and calls_wait:
                # every callee opens with s_waitcnt lgkmcnt(0) (checked in check_library), before it
                # touches a register: the call retires the loads in flight like a wait
                amb |= {x for x, (c, _) in pend.items() if c >= 2}
                pend = {}
        out = (pend, frozenset(amb))
        for j in succ[i]:
            nj = join(IN[j], out)
            if IN[j] is None or nj[0] != IN[j][0] or nj[1] != IN[j][1]:
                IN[j] = nj
                work.append(j)
    return sorted(findings.values())


def check_library(lib, func_filter="_ZN2rt"):
    text = disassemble(lib)
    funcs = parse_functions(text)
    # device functions (they return with s_setpc): does every one open with a full lgkm wait?
    callees = [n for n, ins in funcs.items() if any(m.startswith("s_setpc") and is_return(o) for _, m, o, _ in ins)]
    calls_wait = all(funcs[n] and lgkm_zero(funcs[n][0][1], funcs[n][0][2]) for n in callees)
    checked, problems = 0, []
    for name, ins in funcs.items():
        if func_filter and func_filter not in name or not ins:
            continue
        checked += 1
        problems += check_function(name, ins, calls_wait)
        problems += check_vmem(name, ins, cfg(name, ins), calls_wait)
    return checked, problems


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "ray-tracing-project_amd", "lib", "librtamd.so"))
    ap.add_argument("--function", default="_ZN2rt")
    a = ap.parse_args()
    checked, problems = check_library(a.lib, a.function)
    for p in problems:
        print(p)
    print(f"{checked} functions checked, {len(problems)} findings")
    sys.exit(1 if problems or checked == 0 else 0)


if __name__ == "__main__":
    main()
