#!/usr/bin/env python3
"""Fold a tools/gpu_profile.sh + tools/gpu_pmc.sh run (gpurun_out/*_<tag>) into
profiles/<tag>_*: HBM traffic and SQ PMC summaries, rocprofv3 kernel stats,
the GPU test log and the bench line (roofline.traffic / valu_issue re-derived
from the new PMC files).  Prints the per-kernel figures DESIGN.md §4 tabulates.
Usage: tools/refresh_profiles.py [tag]  (DESIGN.md §4 is edited by hand from its output)"""
import csv
import json
import shutil
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

tag = next((a for a in sys.argv[1:] if not a.startswith("--")), "r01")
O, P = ROOT / "gpurun_out", ROOT / "profiles"
subprocess.run([sys.executable, str(ROOT / "tools/pmc_summary.py"), str(O / f"pmcf_{tag}"),
                str(O / f"pmcw_{tag}"), "512", str(P / f"{tag}_hbm_traffic.json")],
               check=True, stdout=subprocess.DEVNULL)
with open(P / f"{tag}_pmc_table.txt", "w") as f:
    subprocess.run([sys.executable, str(ROOT / "tools/pmc_table.py"), "--json",
                    str(P / f"{tag}_pmc.json"), str(O / f"pmcA_{tag}"), str(O / f"pmcB_{tag}")],
                   check=True, stdout=f)
shutil.copy(O / f"prof_{tag}" / "run_kernel_stats.csv", P / f"{tag}_kernel_stats.csv")
if (O / f"tests_{tag}.log").exists():
    shutil.copy(O / f"tests_{tag}.log", P / f"{tag}_gpu_tests.log")

b = json.loads((O / f"bench_{tag}.json").read_text())
r = b["roofline"]
bl = b["config"]["frames_per_launch"]  # the PMC files are per 512-frame launch, scaled
r["traffic"], _ = bench.measured_traffic(r["kernel"], bl)
vi = bench.valu_issue(r["kernel"], bl, r["ms_per_launch"])
if vi is not None:  # re-derived from the new PMC files
    rate = vi["valu_instr_per_launch"] / (r["ms_per_launch"] * 1e-3) / 1e9
    r["valu"] = dict(r.get("valu", {}), achieved=rate, frac=rate / bench.VALU_PEAK_G,
                     issue_bound=vi)
(P / f"{tag}_bench.json").write_text(json.dumps(b))
print(f"value {b['value']:.0f} frames/s, {b['ms_per_step']:.3f} ms/step, cpu {b['cpu_baseline']['value']:.1f}")
print(f"roofline {r['kernel']} {r['achieved']:.0f} GB/s frac {r['frac']:.4f} "
      f"{r['ms_per_launch']:.3f} ms/launch valu frac {r.get('valu', {}).get('frac')}")

agg = {}
for x in csv.DictReader(open(P / f"{tag}_kernel_stats.csv")):
    n = x["Name"].split("(")[0].replace("void ", "").split("<")[0]
    a = agg.setdefault(n, [0, 0.0])
    a[0] += int(x["Calls"])
    a[1] += float(x["TotalDurationNs"])
sc = [1.0]
for _ in range(7):
    sc.append(float(np.float32(sc[-1] * 1.2)))
alg = bench.algorithmic_bytes(1241, 376, np.float32(sc), 8, b["config"]["mean_keypoints_per_frame"], 5000)
h = json.loads((P / f"{tag}_hbm_traffic.json").read_text())["kernels"]
pm = json.loads((P / f"{tag}_pmc.json").read_text())["kernels"]
# dispatches per extraction call, from the trace itself: k_pyr_resize runs
# nlevels-1 launches, k_fast_cells two (level 0 on the side stream, then levels
# >= 1); the PMC passes run FAST inline (one dispatch), so their per-dispatch
# counters are already per call
calls = {k: agg[k][0] / agg["k_orient_desc"][0] for k in agg}
tb = json.loads((O / f"prof_{tag}.json").read_text())["config"]["frames_per_launch"]
for k in [k for k in ["k_pyr_resize", "k_blur_levels", "k_fast_band", "k_fast_cells", "k_octree",
                      "k_orient_desc"] if k in agg and k in pm]:
    n_launch = round(calls[k])
    ms = agg[k][1] / agg[k][0] / 1e6 * n_launch
    a = alg[k] * tb  # the trace run's frames per launch
    t = h[k]["traffic_bytes"] * (7 if k == "k_pyr_resize" else 1) * tb / 512
    d = pm[k]
    w = d["SQ_WAVE_CYCLES"]
    print(f"{k:16s} {ms:.3f} ms/call ({n_launch} dispatches)  {a / ms / 1e6:6.0f} GB/s  "
          f"frac {a / ms / 1e6 / 8000:.3f}  traffic/alg {t / a:.2f}  wait/inst/active "
          f"{100 * d['SQ_WAIT_ANY'] / w:.0f}/{100 * d['SQ_WAIT_INST_ANY'] / w:.0f}/"
          f"{100 * d['SQ_ACTIVE_INST_ANY'] / w:.0f} %  valu {d['SQ_INSTS_VALU']:.3g}")
