#!/usr/bin/env python3
"""Summarise rocprofv3 output databases (kernel-trace stats + PMC counters) into a text file.

usage: prof_summary.py <out.txt> [--trace DIR] [--pmc DIR ...] [--note TEXT] [--traffic-json OUT --workload W]
       prof_summary.py --from-txt SUMMARY.txt --traffic-json OUT --workload W
--traffic-json writes the per-kernel HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) that bench.py
reports as roofline.traffic for the same workload.
FETCH_SIZE is doubled for the byte estimate: on gfx950 it reports half the bytes of a wide
coalesced read (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.
"""
import argparse
import glob
import sqlite3
from collections import defaultdict


def dbs(d):
    return sorted(glob.glob(f"{d}/**/*.db", recursive=True))


def short(name, n=90):
    name = name.replace("(anonymous namespace)::", "")
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--trace", default=None)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--note", default="")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--from-txt", default=None)
    a = ap.parse_args()
    if a.from_txt:
        write_traffic(open(a.from_txt).read().splitlines(), a.from_txt, a.traffic_json, a.workload)
        return
    lines = []
    if a.note:
        lines += [a.note, ""]
    if a.trace:
        for f in dbs(a.trace):
            c = sqlite3.connect(f)
            lines.append(f"== kernel trace stats ({f.split('gpurun_out/')[-1]})")
            lines.append(f"{'kernel':92s} {'calls':>6s} {'total_ms':>12s} {'avg_ms':>10s} {'pct':>6s}")
            for name, calls, tot, avg, pct in c.execute("select * from top_kernels"):
                lines.append(f"{short(name):92s} {calls:6d} {tot / 1e3:12.1f} {avg / 1e3:10.2f} {pct:6.2f}")
            rows = list(c.execute(
                "select name, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, scratch_size, grid_x, workgroup_x "
                "from kernels where name like '%k_%' group by name"))
            for r in rows:
                lines.append(f"   resources {short(r[0], 60)}: vgpr {r[1]} agpr {r[2]} sgpr {r[3]} lds {r[4]} "
                             f"scratch {r[5]} grid {r[6]} wg {r[7]}")
            lines.append("")
    for d in a.pmc:
        for f in dbs(d):
            c = sqlite3.connect(f)
            agg = defaultdict(list)
            for name, counter, value, dur in c.execute(
                    "select kernel_name, counter_name, value, duration from counters_collection"):
                agg[(name, counter)].append((value, dur))
            lines.append(f"== PMC ({f.split('gpurun_out/')[-1]})")
            for (name, counter), vals in sorted(agg.items()):
                if "(anonymous namespace)::k_" not in name:
                    continue
                v = sum(x for x, _ in vals) / len(vals)
                extra = ""
                if counter == "FETCH_SIZE":
                    extra = f"  -> est. HBM read {2 * v * 1024 / 1e6:.2f} MB/launch (x2 gfx950 correction)"
                if counter == "WRITE_SIZE":
                    extra = f"  -> HBM write {v * 1024 / 1e6:.2f} MB/launch"
                lines.append(f"{short(name, 60):60s} {counter:12s} avg {v:14.2f} KB over {len(vals)} launches{extra}")
            lines.append("")
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if a.traffic_json:
        write_traffic(lines, a.out, a.traffic_json, a.workload)


def write_traffic(lines, source, out, workload):
    """Per-kernel HBM bytes per launch from the summary's PMC lines -> JSON for bench.py."""
    import json
    import re
    kern = {}
    for ln in lines:
        m = re.match(r"^(?:void )?(k_\w+)[<(].*(?:est\. HBM read|HBM write) ([0-9.]+) MB/launch", ln)
        if not m:
            continue
        key = "read" if "HBM read" in ln else "write"
        kern.setdefault(m.group(1), {})[key] = float(m.group(2)) * 1e6
    json.dump({"workload": workload, "source": source, "unit": "bytes per launch",
               "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE, separate passes",
               "kernels": kern}, open(out, "w"), indent=1)
    print(f"wrote {out}: {len(kern)} kernels")


if __name__ == "__main__":
    main()
