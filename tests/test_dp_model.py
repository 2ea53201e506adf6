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
    assert d["best"]["mode"] == "all-reduce"
