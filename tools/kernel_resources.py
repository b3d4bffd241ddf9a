#!/usr/bin/env python3
"""Kernel resource summary of the last `make` (build/kernels/*.o.ru, written
by -Rpass-analysis=kernel-resource-usage): per kernel VGPRs, AGPRs, scratch
bytes per lane and occupancy; kernels that spill to scratch are listed
first. A spill in a hot kernel is memory traffic and latency in its inner
loop (round 6: spf_lds_route_kernel's 44 B/lane cost C3 4 %).
  python tools/kernel_resources.py [--all] [build/kernels/*.o.ru ...]"""
import glob
import re
import subprocess
import sys

FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "occ", "TotalSGPRs": "sgpr"}


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def parse(path):
    rows, cur = [], None
    for ln in open(path, errors="replace"):
        m = re.search(r"remark: Function Name: (\S+)", ln)
        if m:
            cur = {"tu": path.split("/")[-1].split(".")[0], "name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+(?:\[[^\]]*\])?): (\d+)", ln)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[FIELDS[m.group(1).strip()]] = int(m.group(2))
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rows = [r for p in (args or sorted(glob.glob("build/kernels/*.o.ru"))) for r in parse(p)]
    for r, d in zip(rows, demangle([r["name"] for r in rows])):
        r["name"] = d
    spill = [r for r in rows if r.get("scratch", 0) > 0]
    print(f"{len(rows)} kernels, {len(spill)} with scratch")
    show = rows if "--all" in sys.argv else spill
    for r in sorted(show, key=lambda r: -r.get("scratch", 0)):
        print(f"  {r.get('scratch', 0):4d} B/lane  vgpr {r.get('vgpr', '?'):>3} agpr "
              f"{r.get('agpr', '?'):>3} occ {r.get('occ', '?')}  {r['tu']}: {r['name'][:110]}")


if __name__ == "__main__":
    main()
