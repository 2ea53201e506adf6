"""tools/dp_exposure_model.py replays the REAL GradReducer bucket plan of ViT-L Jumbo-MAE (CPU, no
process group): the plan behind README's reducer / bucket-size decision."""

import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_exposure_model_bucket_plan(tmp_path):
    import dp_exposure_model as M

    out = tmp_path / "m.json"
    M.main(["--world", "8", "--bucket-mb", "64", "--json", str(out)])
    d = json.loads(out.read_text())
    rows = {r["mode"]: r for r in d["rows"]}
    ar, z1 = rows["all-reduce"], rows["zero1"]
    # one ViT-L encoder layer (50 MB) per 64 MiB bucket, decoder layers grouped, one bucket per
    # jumbo-MLP kernel (README "Reducer and bucket size at N = 8")
    assert ar["buckets"] == 31
    # ZeRO-1 cuts each oversized jumbo bucket into PARTIAL_SUB sub-buckets (+ snapped boundaries)
    assert z1["buckets"] > ar["buckets"]
    # all-reduce finishes later than the reduce-scatters but the step waits less (the master
    # all-gather runs after the update): the documented default
    assert ar["reduce_done_after_backward_ms"] > z1["reduce_done_after_backward_ms"]
    assert 0 < ar["wait_after_backward_ms"] < z1["wait_after_backward_ms"]
    # ZeRO-1 gathering the bf16 shadow (2 B per parameter) waits less than the fp32-master gather
    assert z1["wait_after_backward_ms"] < rows["zero1-fp32gather"]["wait_after_backward_ms"]
    assert z1["comm_ms"] < rows["zero1-fp32gather"]["comm_ms"]
    # a bf16 reduction halves the reduced bytes (modelled; the fp32 reduction stays the default)
    assert rows["all-reduce-bf16"]["comm_ms"] < ar["comm_ms"]
    fp32 = [r for r in d["rows"] if r["mode"] in ("all-reduce", "zero1", "zero1-fp32gather")]
    assert min(fp32, key=lambda r: r["wait_after_backward_ms"])["mode"] == "all-reduce"


def test_exposure_model_reads_bench_calibration(tmp_path):
    """--sweep takes bench.py's own multi-GPU JSON line (its "collective_sweep" calibration rows)."""
    import dp_exposure_model as M

    rows = [{"size_mb": mb, "bytes": int(mb * 2**20), "world": 8, "allreduce_busbw_GBs": bw}
            for mb, bw in ((8.0, 120.0), (48.0, 260.0), (64.0, 280.0), (288.0, 310.0))]
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"parsed": {"metric": "x", "collective_sweep": rows}}))
    out = tmp_path / "m.json"
    M.main(["--world", "8", "--bucket-mb", "64", "--sweep", str(bench), "--json", str(out)])
    d = json.loads(out.read_text())
    assert d["assumptions"]["sweep"] == str(bench)
    assert all(r["comm_ms"] > 0 for r in d["rows"])
