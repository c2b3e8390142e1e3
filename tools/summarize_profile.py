"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-counter mean over the render-kernel dispatches + derived figures
HBM traffic follows /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide streaming reads, so it is doubled;
both are collected in separate passes.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


MAX_CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md: max engine clock


def issue_block(out, mean, avg_ns, clock=None):
    """Clock and issue roofline of one kernel. The clock the issue fractions use:
    * the in-kernel clock when measured (clock = tools/kernel_clock.py's record: median over the waves of a
      timeline frame of the same workload of delta s_memtime / delta s_memrealtime x 100 MHz, the method of
      MI355X_MICROARCH.md "DVFS give-back" item 6);
    * else GRBM_GUI_ACTIVE / 8 / the trace's kernel duration, capped at the chip's 2.4 GHz: that quotient counts
      the counter window, which on dispatches shorter than ~0.3 ms is longer than the kernel, so it reads high
      (C2's 70-us kernel: 2.88 GHz) -- kept as grbm_quotient_GHz, not used above the cap.
    Issue capacity per cycle: one wave64 VALU instruction per 2 cycles per SIMD (4 SIMDs per CU), one SALU / one
    SMEM instruction per cycle per CU (MI355X_MICROARCH.md); the fractions are over clock x kernel duration.
    SQ_WAVE_CYCLES and the SQ_WAIT / ACTIVE counters are in quad-cycles."""
    if "GRBM_GUI_ACTIVE" not in mean or not avg_ns:
        return
    q = mean["GRBM_GUI_ACTIVE"] / 8 / avg_ns
    out["grbm_quotient_GHz"] = round(q, 4)
    if clock and clock.get("clock_GHz"):
        clk, src = float(clock["clock_GHz"]), "in-kernel: median over waves of d(s_memtime) / d(s_memrealtime) x 100 MHz (" + \
            str(clock.get("what", "timeline frame")) + ")"
    elif q > MAX_CLOCK_GHZ:
        clk, src = MAX_CLOCK_GHZ, f"GRBM_GUI_ACTIVE / 8 / kernel duration = {q:.2f} GHz reads above the 2.4 GHz maximum " \
            "(counter window longer than a short dispatch): capped at 2.4, so the issue fractions are lower bounds"
    else:
        clk, src = q, "GRBM_GUI_ACTIVE / 8 / kernel duration"
    out["effective_clock_GHz"] = clk
    out["clock_source"] = src
    cyc = avg_ns * clk
    issue = {"clock_GHz": round(clk, 3), "kernel_ns": round(avg_ns, 1)}
    if "SQ_INSTS_VALU" in mean:
        issue["valu_per_launch"] = mean["SQ_INSTS_VALU"]
        issue["valu_frac"] = round(mean["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 4)
    if "SQ_INSTS_SALU" in mean:
        issue["salu_per_launch"] = mean["SQ_INSTS_SALU"]
        issue["salu_frac"] = round(mean["SQ_INSTS_SALU"] / (256 * cyc), 4)
    if "SQ_INSTS_SMEM" in mean:
        issue["smem_frac"] = round(mean["SQ_INSTS_SMEM"] / (256 * cyc), 4)
    if "SQ_WAVE_CYCLES" in mean:
        issue["mean_resident_waves_per_simd"] = round(4 * mean["SQ_WAVE_CYCLES"] / (1024 * cyc), 2)
        for k, name in (("SQ_WAIT_ANY", "wave_cycles_waiting"), ("SQ_ACTIVE_INST_ANY", "wave_cycles_issuing"),
                        ("SQ_WAIT_INST_ANY", "wave_cycles_issue_stalled")):
            if k in mean:
                issue[name] = round(mean[k] / mean["SQ_WAVE_CYCLES"], 4)
    out["issue"] = issue
    if "valu_frac" in issue and "wave_cycles_waiting" in issue:
        out["limiter"] = (f"latency: waves wait on memory (s_waitcnt) {100 * issue['wave_cycles_waiting']:.0f}% "
                          f"of their cycles and issue in {100 * issue.get('wave_cycles_issuing', 0):.0f}%; "
                          f"VALU issue at {100 * issue['valu_frac']:.0f}% and SALU at "
                          f"{100 * issue.get('salu_frac', 0):.0f}% of peak; HBM at "
                          f"{100 * out.get('hbm_bytes_per_launch', 0) / avg_ns / 8000:.1f}% of 8 TB/s")


def refresh(paths):
    """Recompute the clock / issue / limiter fields of committed profiles/*_pmc.json from their stored counters
    (the clock rule above; files without GRBM_GUI_ACTIVE are left as they are)."""
    for p in paths:
        d = json.load(open(p))
        mean, avg_ns = d.get("counters_mean_per_dispatch") or {}, d.get("avg_kernel_ns_trace")
        if "GRBM_GUI_ACTIVE" not in mean or not avg_ns:
            continue
        for k in ("issue", "limiter", "effective_clock_GHz", "clock_source", "grbm_quotient_GHz"):
            d.pop(k, None)
        issue_block(d, mean, avg_ns, d.get("kernel_clock"))
        json.dump(d, open(p, "w"), indent=1)
        print(os.path.basename(p), d["effective_clock_GHz"], d.get("grbm_quotient_GHz"))


def main(tag, prof=os.path.join(ROOT, "gpurun_out", "prof"), kernel=None):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    if kernel is None:  # the bench line's dominant kernel, non-counting instantiation
        try:
            bl = json.loads(open(os.path.join(prof, "trace_bench.json")).read().strip().splitlines()[-1])
            kernel = bl["roofline"]["kernel"] + "<false"
        except Exception:
            kernel = "k_primary_fused<false"
    stats_src = os.path.join(prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats_src)):
        if "::" + kernel in r["Name"]:
            avg_ns = float(r["AverageNs"])
    counters = defaultdict(list)
    for d in sorted(os.listdir(prof)):
        f = os.path.join(prof, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            for r in csv.DictReader(open(f)):
                if "::" + kernel in r["Kernel_Name"]:
                    counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in counters.items()}
    out = {"kernel": kernel, "avg_kernel_ns_trace": avg_ns, "counters_mean_per_dispatch": mean,
           "dispatches_per_counter": {k: len(v) for k, v in counters.items()}}
    bench = os.path.join(prof, "trace_bench.json")
    if os.path.exists(bench):
        try:
            out["bench_line_under_trace"] = json.loads(open(bench).read().strip().splitlines()[-1])
        except Exception:
            pass
    # the same average restricted to the bench's timed launches, which is what the bench line's HIP-event
    # kernel_ms measures. Dispatch order of this kernel (the counting run, the parity frame and the end-to-end
    # frames use other instantiations or are off under profile.sh): the prewarm frames (round 5), the warm-up
    # frames, the timed steps, then the 20 isolated frames of bench.isolated_kernel_ms -- so the timed steps
    # are the K dispatches before the last 20
    trace_csv = os.path.join(prof, "trace", "run_kernel_trace.csv")
    bl = out.get("bench_line_under_trace")
    if bl and os.path.exists(trace_csv):
        rows = [r for r in csv.DictReader(open(trace_csv)) if "::" + kernel in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        k, iso = int(bl["steps"]), 20
        sel = rows[len(rows) - iso - k:len(rows) - iso] if len(rows) >= iso + k else []
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]
        if len(d) == k:
            out["avg_kernel_ns_timed_region"] = sum(d) / k
            rl = bl.get("roofline") or {}
            out["bench_kernel_ns_hip_events"] = (rl.get("kernel_ms_isolated") or rl.get("kernel_ms") or 0) * 1e6
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        fetch = 2.0 * mean["FETCH_SIZE"] * 1024
        write = mean["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = fetch + write
        out["hbm_read_bytes_per_launch_corrected"] = fetch
        out["hbm_write_bytes_per_launch"] = write
        if avg_ns:
            out["hbm_GBps"] = (fetch + write) / avg_ns
    clock = None
    cf = os.path.join(prof, "kernel_clock.json")  # tools/kernel_clock.py, written by tools/profile.sh
    if os.path.exists(cf):
        try:
            clock = json.load(open(cf))
        except ValueError:
            clock = None
    if clock:
        out["kernel_clock"] = clock
    issue_block(out, mean, avg_ns, clock)
    if "SQ_WAVE_CYCLES" in mean:
        wc = mean["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in mean:
                out[f"frac_{k}"] = mean[k] / wc
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        out["l2_hit_rate"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
    if "SQ_WAVES" in mean:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD"):
            if k in mean:
                out[f"{k}_per_wave"] = mean[k] / mean["SQ_WAVES"]
    out["tag"] = tag
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    # RT_PROFILE_LATEST: 1 (default) the headline workload's profile -> pmc_latest.json; c5 / c2 the bench
    # line's C5 / C2 sub-line profile -> pmc_latest_c5.json / pmc_latest_c2.json; 0 a side profile only
    latest = os.environ.get("RT_PROFILE_LATEST", "1")
    if latest != "0":
        name = "pmc_latest.json" if latest == "1" else f"pmc_latest_{latest}.json"
        json.dump(out, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "bench_line_under_trace"}, indent=1))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--refresh"]:
        refresh(sys.argv[2:])
    else:
        main(*sys.argv[1:])
