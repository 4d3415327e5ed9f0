#!/usr/bin/env python3
"""Summarise a scripts/prof_run.sh output directory (rocprofv3 databases) into a text file.

usage: prof_summary.py <run dir> <out.txt> [--note TEXT] [--traffic-json profiles/pmc_traffic.json --workload KEY]
       prof_summary.py --merge <box pmc_traffic.json> profiles/pmc_traffic.json

Sections: the kernel-trace stats (calls, total, average per launch, resources), then per kernel the PMC
counters averaged over launches with derived ratios:
  HBM bytes    FETCH_SIZE (KB) x 2 -- on gfx950 it reports half the bytes of a wide coalesced read
               (MI355X_MICROARCH.md, HBM section) -- and WRITE_SIZE (KB) as is
  VALU busy    SQ_ACTIVE_INST_VALU / (SQ_BUSY_CYCLES x 4 SIMDs ... ) is not comparable across kernels,
               so the ratios given are per wave: VALU instructions per wave, wait and active cycle shares
               of SQ_WAVE_CYCLES
--traffic-json merges this workload's per-kernel HBM bytes per launch into the JSON bench.py reads
(roofline.traffic), keyed by the workload string bench.py prints (config/pipeline/mode/side).
"""
import argparse
import glob
import json
import sqlite3
from collections import defaultdict
from pathlib import Path


def dbs(d):
    return sorted(glob.glob(f"{d}/**/*.db", recursive=True))


def short(name, n=80):
    name = name.replace("(anonymous namespace)::", "")
    return name if len(name) <= n else name[: n - 3] + "..."


def kname(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("<")[0]


def trace_section(d):
    lines = []
    for f in dbs(d):
        c = sqlite3.connect(f)
        lines.append(f"== kernel trace stats ({Path(f).parent.name})")
        lines.append(f"{'kernel':82s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'pct':>6s}")
        for name, calls, tot, avg, pct in c.execute("select * from top_kernels"):
            lines.append(f"{short(name):82s} {calls:6d} {tot / 1e3:10.3f} {avg / 1e3:9.4f} {pct:6.2f}")
        for r in c.execute("select name, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, scratch_size, grid_x, "
                           "workgroup_x from kernels where name like '%k_%' group by name"):
            lines.append(f"   resources {short(r[0], 60)}: vgpr {r[1]} agpr {r[2]} sgpr {r[3]} lds {r[4]} "
                         f"scratch {r[5]} grid {r[6]} wg {r[7]}")
        lines.append("")
    return lines


def pmc(d):
    """{kernel: {counter: mean value per launch}} over every PMC database under d (trace excluded)."""
    agg = defaultdict(lambda: defaultdict(list))
    for f in dbs(d):
        if Path(f).parent.name == "trace":
            continue
        c = sqlite3.connect(f)
        try:
            rows = list(c.execute("select kernel_name, counter_name, value from counters_collection"))
        except sqlite3.OperationalError:
            continue
        for name, counter, value in rows:
            # bench.py's one counted frame (k_trace<..., kCount = true>) is not the timed kernel
            if "k_" in name and not ("k_trace<" in name and ", true>(" in name):
                agg[kname(name)][counter].append(value)
    return {k: {cn: sum(v) / len(v) for cn, v in cs.items()} for k, cs in agg.items()}


def pmc_section(p):
    lines = ["== PMC counters (mean per launch; separate rocprofv3 passes)"]
    for k in sorted(p):
        c = p[k]
        lines.append(f"-- {k}")
        for cn in sorted(c):
            lines.append(f"   {cn:22s} {c[cn]:18.1f}")
        if "FETCH_SIZE" in c:
            lines.append(f"   => HBM read  {2 * c['FETCH_SIZE'] * 1024 / 1e6:10.2f} MB/launch (FETCH_SIZE KB x2, gfx950)")
        if "WRITE_SIZE" in c:
            lines.append(f"   => HBM write {c['WRITE_SIZE'] * 1024 / 1e6:10.2f} MB/launch (WRITE_SIZE KB)")
        if c.get("SQ_WAVES"):
            w = c["SQ_WAVES"]
            lines.append(f"   => per wave: VALU insts {c.get('SQ_INSTS_VALU', 0) / w:9.1f}"
                         + (f"  SALU {c['SQ_INSTS_SALU'] / w:8.1f}" if "SQ_INSTS_SALU" in c else "")
                         + (f"  SMEM {c['SQ_INSTS_SMEM'] / w:7.1f}" if "SQ_INSTS_SMEM" in c else "")
                         + (f"  LDS {c['SQ_INSTS_LDS'] / w:7.1f}" if "SQ_INSTS_LDS" in c else "")
                         + (f"  VMEM rd {c['SQ_INSTS_VMEM_RD'] / w:6.1f}" if "SQ_INSTS_VMEM_RD" in c else ""))
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            parts = [f"{n} {100 * c[cn] / wc:5.1f}%" for n, cn in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                                                                    ("active_any", "SQ_ACTIVE_INST_ANY"),
                                                                    ("active_valu", "SQ_ACTIVE_INST_VALU")) if cn in c]
            lines.append("   => share of wave cycles: " + "  ".join(parts))
        if c.get("SQ_BUSY_CYCLES") and c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_WAVES"):
            # SQ_ACTIVE_INST_VALU sums per-wave VALU-active cycles; over the SIMD-cycles available
            # (busy cycles of the SQ x 4 SIMDs x CUs per SQ is not exposed) it is only a relative figure
            pass
    lines.append("")
    return lines


def write_traffic(p, source, out, workload):
    kern = {}
    for k, c in p.items():
        e = {}
        if "FETCH_SIZE" in c:
            e["read"] = 2 * c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            e["write"] = c["WRITE_SIZE"] * 1024
        # issue counts per launch (bench.py's issue roof for kernels without a flop model, e.g. k_traverse)
        for cn, key in (("SQ_INSTS_VALU", "valu_insts"), ("SQ_INSTS_SALU", "salu_insts"), ("SQ_INSTS_SMEM", "smem_insts"),
                        ("SQ_WAVES", "waves")):
            if cn in c:
                e[key] = c[cn]
        if e:
            kern[k] = e
    path = Path(out)
    d = json.loads(path.read_text()) if path.exists() else {}
    d.setdefault("workloads", {})
    d["unit"] = "HBM bytes per launch"
    d["workloads"][workload] = {"source": source, "kernels": kern,
                                "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE, separate passes; "
                                          "SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_INSTS_SMEM / SQ_WAVES per launch from the SQ passes"}
    path.write_text(json.dumps(d, indent=1) + "\n")
    print(f"wrote {out}: {workload}: {len(kern)} kernels")


def merge(src, dst):
    """Merge the workloads of a box-side pmc_traffic.json into the committed one."""
    d = json.loads(Path(dst).read_text()) if Path(dst).exists() else {"unit": "HBM bytes per launch"}
    d.setdefault("workloads", {}).update(json.loads(Path(src).read_text())["workloads"])
    Path(dst).write_text(json.dumps(d, indent=1) + "\n")


def main():
    import sys
    if len(sys.argv) == 4 and sys.argv[1] == "--merge":
        merge(sys.argv[2], sys.argv[3])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("rundir")
    ap.add_argument("out")
    ap.add_argument("--note", default="")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--workload", default=None)
    ap.add_argument("--source", default=None, help="path recorded as the workload's source (the committed copy)")
    a = ap.parse_args()
    lines = [a.note, ""] if a.note else []
    lines += trace_section(f"{a.rundir}/trace")
    p = pmc(a.rundir)
    lines += pmc_section(p)
    Path(a.out).write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
    if a.traffic_json:
        write_traffic(p, a.source or a.out, a.traffic_json, a.workload)


if __name__ == "__main__":
    main()
