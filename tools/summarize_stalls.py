"""Summarise a tools/pmc_stalls.sh run: per hlgs kernel, every counter averaged per launch, plus derived busy /
stall ratios.  Conventions (MI355X_MICROARCH.md, PMC and cycle-constant sections):
  - SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles summed over waves: their ratios are the share of
    resident-wave time spent issuing / parked / issue-stalled (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES);
  - GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = GRBM_GUI_ACTIVE / 8;
  - a wave64 VALU instruction occupies a SIMD-32 for 2 cycles, so the VALU issue ceiling is
    1024 SIMDs x 1 instr / 2 cycles: valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 * kernel_cycles);
  - fetch = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE, both KiB.

    python tools/summarize_stalls.py gpurun_out/stall profiles/r02/stalls.json
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, CUS = 1024, 256


def load(src):
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for path in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
        per_dispatch = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "hlgs::" not in name:
                continue
            key = (name, r["Dispatch_Id"])
            c = r["Counter_Name"]
            per_dispatch[key][c] = per_dispatch[key].get(c, 0.0) + float(r["Counter_Value"])
        for (name, _), cs in per_dispatch.items():
            for c, v in cs.items():
                cnt[name][c].append(v)
    for path in glob.glob(os.path.join(src, "p1", "run_kernel_trace.csv")):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "hlgs::" in name:
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return cnt, dur


def main(src, dst):
    cnt, dur = load(src)
    out = {}
    for k, cs in sorted(cnt.items()):
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(counters={c: round(v, 1) for c, v in sorted(a.items())}, launches=len(next(iter(cs.values()))))
        if dur.get(k):
            d["pmc_pass_us"] = round(1e6 * sum(dur[k]) / len(dur[k]), 2)
        g = a.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8
            d["kernel_cycles"] = round(cyc)
            if d.get("pmc_pass_us"):
                d["clock_GHz"] = round(cyc / (d["pmc_pass_us"] * 1e3), 3)
            if "SQ_INSTS_VALU" in a:
                d["valu_issue_frac"] = round(2 * a["SQ_INSTS_VALU"] / (SIMDS * cyc), 4)
            if "SQ_INSTS_SALU" in a:
                d["salu_per_cu_cycle"] = round(a["SQ_INSTS_SALU"] / (CUS * cyc), 4)
            if "SQ_INSTS_LDS" in a:
                d["lds_instr_per_cu_cycle"] = round(a["SQ_INSTS_LDS"] / (CUS * cyc), 4)
            if "SQ_WAVE_CYCLES" in a:
                d["waves_per_simd"] = round(4 * a["SQ_WAVE_CYCLES"] / (SIMDS * cyc), 3)
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            d["share_of_wave_time"] = {n: round(a[c] / wc, 4) for n, c in
                                       (("issuing_any", "SQ_ACTIVE_INST_ANY"), ("issuing_valu", "SQ_ACTIVE_INST_VALU"),
                                        ("issuing_salu", "SQ_ACTIVE_INST_SCA"), ("issuing_lds", "SQ_ACTIVE_INST_LDS"),
                                        ("issuing_vmem", "SQ_ACTIVE_INST_VMEM"), ("issuing_misc", "SQ_ACTIVE_INST_MISC"),
                                        ("parked_waitcnt_barrier", "SQ_WAIT_ANY"),
                                        ("issue_stalled", "SQ_WAIT_INST_ANY"), ("lds_issue_stalled", "SQ_WAIT_INST_LDS"))
                                       if c in a}
        if a.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_share"] = round(a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in a or "WRITE_SIZE" in a:
            d["fetch_bytes"] = round(2 * 1024 * a.get("FETCH_SIZE", 0.0))
            d["write_bytes"] = round(1024 * a.get("WRITE_SIZE", 0.0))
        out[k] = d
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from summarize_profile import build_identity
    json.dump(dict(note=__doc__.strip().splitlines()[0] + " (see tools/summarize_stalls.py for conventions)",
                   build=build_identity(), kernels=out), open(dst, "w"), indent=1)
    for k, d in out.items():
        if "blend" in k or "preprocess" in k:
            print(k, json.dumps({x: d.get(x) for x in ("pmc_pass_us", "clock_GHz", "valu_issue_frac", "salu_per_cu_cycle",
                                                       "waves_per_simd", "share_of_wave_time", "lds_bank_conflict_share",
                                                       "fetch_bytes", "write_bytes")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
