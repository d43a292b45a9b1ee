#!/usr/bin/env python3
"""Summarise gpurun_out/prof_<tag>/ (from tools/profile_bench.sh) into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, as produced), profiles/<tag>_summary.md and
profiles/<tag>_traffic.json: per-kernel average duration and HBM traffic per launch from the PMC
passes.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64-B units for
128-B requests, i.e. it reads 1/2 of the bytes of wide coalesced reads -> traffic uses
2 * FETCH_SIZE + WRITE_SIZE (both reported in KiB by rocprofv3)."""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


def pmc(path, counter):
    agg = collections.defaultdict(list)
    per_disp = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per_disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
    for d, v in per_disp.items():
        agg[names[d]].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    vpath = os.path.join(src, "valu", "run_counter_collection.csv")
    valu = pmc(vpath, "SQ_INSTS_VALU") if os.path.exists(vpath) else {}
    rows = []
    total = sum(float(r["TotalDurationNs"]) for r in stats)
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"])):
        k = short(r["Name"])
        f = fetch.get(k)
        w = write.get(k)
        traffic = (2 * f + w) * 1024 if f is not None and w is not None else None
        v = valu.get(k)
        # VALU issue roofline: a wave64 VALU op occupies its SIMD 2 cycles (32 lanes/cycle); 1024 SIMDs at
        # 2.4 GHz issue at most 1.2288e12 wave-instructions/s chip-wide
        vfrac = v / (float(r["AverageNs"]) * 1e-9 * 1024 * 2.4e9 / 2) if v else None
        rows.append(dict(kernel=k, calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                         pct=100 * float(r["TotalDurationNs"]) / total, fetch_kib=f, write_kib=w,
                         hbm_bytes_per_launch=traffic, valu_insts=v, valu_issue_frac=vfrac))
    json.dump({"tag": tag, "kernels": rows}, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary `{tag}`\n\nCommand: `tools/profile_bench.sh {tag}` = rocprofv3 over "
                 "`python3 bench.py --no-cpu-baseline --no-sub` (the default 30 timed + 20 warmup steps of the bench line, sub-records skipped; cfg3: 200k splats, 1e7 texels, "
                 "800x800, full train step).\nTraffic = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 per launch "
                 "(separate --pmc passes; gfx950 FETCH_SIZE halving corrected).\nVALU issue = SQ_INSTS_VALU "
                 "per launch / (avg duration x 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction).\n\n")
        fh.write("| kernel | calls | avg us | % time | HBM MB/launch | VALU instr/launch | VALU issue |\n"
                 "|---|---|---|---|---|---|---|\n")
        for r in rows[:25]:
            t = "" if r["hbm_bytes_per_launch"] is None else f"{r['hbm_bytes_per_launch'] / 1e6:.1f}"
            v = "" if not r.get("valu_insts") else f"{r['valu_insts']:.3g}"
            vf = "" if not r.get("valu_issue_frac") else f"{100 * r['valu_issue_frac']:.0f}%"
            fh.write(f"| {r['kernel'][:60]} | {r['calls']} | {r['avg_us']:.1f} | {r['pct']:.1f} | {t} | {v} | {vf} |\n")
    print(open(os.path.join(dst, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
