"""The measurement helpers behind bench.py's `roofline.traffic`:
scripts/pmc_traffic.py turns rocprofv3 --pmc counter CSVs into bytes per
launch (one kernel, medians) or per step (every engine kernel of N steps
summed), with the gfx950 FETCH_SIZE correction (fetched = 2 x FETCH_SIZE KB;
profiles/r02/c4/fetch_calibration.json). Synthetic CSVs, no GPU."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "scripts", "pmc_traffic.py")


def _write_pass(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "p_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _run(args):
    out = subprocess.run([sys.executable, TOOL, *args], capture_output=True, text=True, check=True)
    return out.stdout


def test_per_launch_median_and_correction(tmp_path):
    k = "void (anonymous namespace)::k_score<1, float, true>(ScoreParams)"
    _write_pass(tmp_path / "f", [{"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE",
                                  "Counter_Value": v} for i, v in enumerate([100.0, 300.0, 200.0])])
    _write_pass(tmp_path / "w", [{"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": "WRITE_SIZE",
                                  "Counter_Value": 50.0} for i in range(3)])
    out = tmp_path / "o.json"
    _run(["c2", "k_score<1, float, true>", str(out), str(tmp_path / "f"), str(tmp_path / "w")])
    r = json.load(open(out))
    assert r["fetch_bytes_corrected"] == 200.0 * 1024 * 2       # median, x2 line correction
    assert r["write_bytes"] == 50.0 * 1024
    assert r["traffic_bytes_per_launch"] == 200.0 * 2048 + 50.0 * 1024


def test_per_step_sum_excludes_runtime_and_named_kernels(tmp_path):
    rows = [
        {"Dispatch_Id": 1, "Kernel_Name": "k_neighbours<1>(NbrParams)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 10.0},
        {"Dispatch_Id": 2, "Kernel_Name": "k_score_wide<1, float, 1024, 10>(ScoreParams)", "Counter_Name": "FETCH_SIZE",
         "Counter_Value": 30.0},
        {"Dispatch_Id": 3, "Kernel_Name": "__amd_rocclr_copyBuffer", "Counter_Name": "FETCH_SIZE", "Counter_Value": 1e6},
        {"Dispatch_Id": 4, "Kernel_Name": "k_topk_dense<float>(DenseTopkParams)", "Counter_Name": "FETCH_SIZE",
         "Counter_Value": 1e6},
    ]
    _write_pass(tmp_path / "f", rows)
    out = tmp_path / "o.json"
    _run(["c5", "step:2:k_topk_dense", str(out), str(tmp_path / "f")])
    r = json.load(open(out))
    assert r["per_step"]["FETCH_SIZE"] == 20.0                    # (10 + 30) / 2 steps
    assert r["traffic_bytes_per_launch"] == 20.0 * 1024 * 2
