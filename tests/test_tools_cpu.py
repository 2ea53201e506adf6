"""CPU checks of the measurement tools whose records the README cites (they run on the GPU box for the
records; here the CPU parts: argument handling, JSON shape, the trace arithmetic)."""

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_augment_bytes_cpu(tmp_path):
    """tools/augment_bytes.py: crop windows drawn as the loader workers draw them; H2D bytes above the
    finished images' (windows carry the filter margin), scratch = rows x 224 x 3 per image."""
    import augment_bytes as A

    out = tmp_path / "a.json"
    s = A.main(["--batch", "16", "--batches", "2", "--json", str(out)])
    d = json.loads(out.read_text())
    assert d["summary"] == s and len(d["rows"]) == 2
    for r in d["rows"]:
        assert r["h2d_bytes"] > 0 and r["tmp_bytes"] == r["tmp_bytes"] // (224 * 3) * 224 * 3
        assert "gpu_transient_peak_bytes" not in r
    assert s["host_images_mb"] * 2 ** 20 == 16 * 3 * 224 * 224
    assert 0.0 <= s["fallback_crop_frac"] <= 1.0


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_overlap_check_counts_overlap(tmp_path):
    """tools/overlap_check.py: H2D copies / augment kernels under model kernels, idle gaps per step."""
    import overlap_check as O

    ks, cs = [], []
    t = 0
    for step in range(4):
        ks.append({"Kernel_Name": "adamw_kernel", "Start_Timestamp": t, "End_Timestamp": t + 1000})
        ks.append({"Kernel_Name": "gemm", "Start_Timestamp": t + 1000, "End_Timestamp": t + 9000})
        ks.append({"Kernel_Name": "rrc_h_kernel", "Start_Timestamp": t + 2000, "End_Timestamp": t + 3000})
        cs.append({"Direction": "HOST_TO_DEVICE", "Start_Timestamp": t + 8000, "End_Timestamp": t + 10000})
        t += 100000  # 90 us idle after each step's kernels
    ks.append({"Kernel_Name": "adamw_kernel", "Start_Timestamp": t, "End_Timestamp": t + 1000})
    kp, cp = tmp_path / "k.csv", tmp_path / "c.csv"
    _trace(kp, ks)
    with open(cp, "w", newline="") as f:
        w = csv.DictWriter(f, ["Direction", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in cs:
            w.writerow(r)
    out = O.main([str(kp), str(cp), "--last", "3"])
    assert out["steps"] == 3 and abs(out["step_ms"] - 0.1) < 1e-9
    assert out["augment_overlapped_frac"] == 1.0
    assert abs(out["h2d_overlapped_frac"] - 0.5) < 1e-9  # 1 of the 2 us copy runs under the GEMM
    # gaps between the window's merged kernel intervals: the one before the closing marker (whose
    # start ends the window) is outside it, so 2 gaps over 3 steps
    assert abs(out["idle_gaps_over_20us_per_step"] - 2 / 3) < 1e-9
    assert abs(out["idle_ms_per_step"] - 2 * 0.091 / 3) < 1e-9
