"""Copy a tools/profile_round.sh run into profiles/<round>/: rocprofv3 kernel stats, the bench JSON line,
and per-launch HBM traffic of every hlgs kernel from the FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB.  On gfx950 FETCH_SIZE counts half the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM section), so fetched bytes are taken as 2 x FETCH_SIZE;
WRITE_SIZE is used as is.  Both count L2->fabric traffic, so Infinity-Cache hits are included.

    python tools/summarize_profile.py gpurun_out/round profiles/r01
"""
import collections
import csv
import json
import os
import shutil
import sys


def build_identity():
    """The profiled library: its hash (hashed here, on the box, from the very file the passes loaded) and the commit
    recorded at build time (hierarchical-lod-gaussians_amd/lib/build_info.json)."""
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "hierarchical-lod-gaussians_amd", "lib", "libhlgs.so")
    info = {}
    try:
        info = json.load(open(os.path.join(os.path.dirname(lib), "build_info.json")))
    except (OSError, ValueError):
        pass
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None
    return dict(lib_sha16=sha, head=info.get("head"), sources_dirty=info.get("sources_dirty"))


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        if "hlgs::" in name:
            vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def launch_timing(trace_csv, bench_line, kernel="k_blend_bwd<false, true, false>"):
    """Durations of one kernel from the kernel trace of the bench command, cut into the phases its JSON line's
    launch_plan names (warm-up, stage-timing pass, timed steps, and the last `evented` timed steps whose launches the
    bench brackets with HIP events), beside the bench's own event time for those launches (roofline.kernel_ms): the
    reconciliation of the event time with the rocprof averages."""
    rows = []
    for r in csv.DictReader(open(trace_csv)):
        if kernel in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    us = [(e - b) / 1e3 for b, e in rows]
    plan = bench_line.get("launch_plan") or {}
    w, st, k, ev = (int(plan.get(x, 0)) for x in ("warmup", "stage_timing", "timed", "evented"))
    st += int(plan.get("settle", 0))  # the clock-settle steps run between the stage pass and the timed steps
    avg = lambda v: round(sum(v) / len(v), 2) if v else None  # noqa: E731
    timed = us[w + st:w + st + k]
    out = dict(kernel=kernel, launches=len(us), all_avg_us=avg(us), warmup_avg_us=avg(us[:w]),
               stage_and_settle_avg_us=avg(us[w:w + st]), settle_steps=int(plan.get("settle", 0)), timed_avg_us=avg(timed), timed_min_us=min(timed) if timed else None,
               timed_max_us=max(timed) if timed else None, evented_avg_us=avg(timed[k - ev:]) if ev else None,
               after_timed_avg_us=avg(us[w + st + k:]),
               bench_event_us=round(1e3 * bench_line["roofline"]["kernel_ms"], 2) if bench_line.get("roofline") else None,
               timed_gaps_us=None)
    if len(rows) >= w + st + k and k > 1:
        seg = rows[w + st:w + st + k]
        out["timed_gaps_us"] = avg([(seg[i + 1][0] - seg[i][1]) / 1e3 for i in range(len(seg) - 1)])
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):  # absent when called on the box before the trace run
        shutil.copy(stats, os.path.join(dst, "bench_kernel_stats.csv"))
    dom = os.path.join(src, "trace", "run_domain_stats.csv")
    if os.path.exists(dom):
        shutil.copy(dom, os.path.join(dst, "bench_domain_stats.csv"))
    plain = os.path.join(src, "bench_plain.log")
    if os.path.exists(plain):  # absent when called on the box before the plain bench run
        line = [l for l in open(plain).read().splitlines() if l.startswith("{")][-1]
        json.loads(line)
        open(os.path.join(dst, "bench_line.json"), "w").write(line + "\n")
    traced = os.path.join(src, "bench_line.log")
    if os.path.exists(traced):
        line = [l for l in open(traced).read().splitlines() if l.startswith("{")][-1]
        open(os.path.join(dst, "bench_line_under_rocprof.json"), "w").write(line + "\n")
        tr = os.path.join(src, "trace", "run_kernel_trace.csv")
        if os.path.exists(tr):
            json.dump(dict(launch_timing(tr, json.loads(line)), build=build_identity()),
                      open(os.path.join(dst, "timing.json"), "w"), indent=1)
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    sqp = os.path.join(src, "sq", "run_counter_collection.csv")
    valu = per_kernel(sqp, "SQ_INSTS_VALU") if os.path.exists(sqp) else {}
    salu = per_kernel(sqp, "SQ_INSTS_SALU") if os.path.exists(sqp) else {}
    lds = per_kernel(sqp, "SQ_INSTS_LDS") if os.path.exists(sqp) else {}
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = 2 * 1024 * fetch.get(k, 0.0)
        w = 1024 * write.get(k, 0.0)
        out[k] = dict(fetch_bytes=round(f), write_bytes=round(w), hbm_bytes=round(f + w),
                      valu_wave_instr=round(valu.get(k, 0.0)), salu_wave_instr=round(salu.get(k, 0.0)),
                      lds_wave_instr=round(lds.get(k, 0.0)))
    json.dump(dict(note="per launch; fetch = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE (KiB -> bytes); "
                        "*_wave_instr = SQ_INSTS_* (wave instructions issued, all CUs)",
                   build=build_identity(), kernels=out), open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
