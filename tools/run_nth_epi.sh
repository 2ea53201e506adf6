# GELU_D / DMUL epilogues on the 2-WG/CU 256x128 kernel (variant 10) vs the default: numerics + microbench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python - > gpurun_out/nth_check.txt 2>&1 <<'PY' || { cat gpurun_out/nth_check.txt; exit 1; }
import torch
from jumbo_mae_tpu_amd.ops import _ext
ext = _ext.load(True)
torch.manual_seed(0)
M, N, K = 3000, 2048, 512
x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16(); w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
b = torch.randn(N, device="cuda") * 0.1
dy = (torch.randn(M, 384, device="cuda") * 0.5).bfloat16(); w2t = (torch.randn(N, 384, device="cuda") * 0.05).bfloat16()
outs = {}
for v in (12, 10):
    ext.gemm_set_variant(v, 8)
    gp, g = ext.gemm_nt(x, w, b, True, False, True)
    db = torch.zeros(N, device="cuda")
    d = ext.gemm_nt_dgelu(dy, w2t, gp, db, True)
    torch.cuda.synchronize()
    outs[v] = (gp, g, d, db)
ext.gemm_set_variant(12, 8)
for a, c in zip(outs[12], outs[10]):
    r = ((a.float() - c.float()).norm() / (c.float().norm() + 1e-12)).item()
    print("rel", r); assert r < 1e-2
print("NTH_OK")
PY
tail -1 gpurun_out/nth_check.txt
for v in 0 10; do
timeout -k 10 200 python tools/gelu_epi_bench.py --rounds 2 --variant $v > gpurun_out/nth_v$v.txt 2>&1 || { cat gpurun_out/nth_v$v.txt; exit 1; }
echo "== variant $v"; grep -v amdgpu gpurun_out/nth_v$v.txt | grep -v "save h\|gelu'(h)"
done
