#!/bin/bash
# Diagnostic builds behind profiles/r6j_attn_bwd_diag.txt, r6o_attn_enc_bwd_diag.txt and r6t_ln_bwd_bytes.txt: a copy of
# the package at a git revision with ONE kernel edited (its outputs are garbage -- timing only), built in-tree under
# _abc/<name> (git-ignored; it travels with the gpurun snapshot, run it with JMAE_ROOT=_abc/<name>).  Run HERE (CPU):
#   bash tools/r6_diag_trees.sh <name> [rev]      names:
#     d1  decoder attention backward (attn_bwd3) without its global loads
#     d2  attn_bwd3 without its compute loop (loads + staging + dK / dV stores)
#     d3  attn_bwd3 loading K and V only          d4  attn_bwd3 loading Q / dO / O only
#     d5  encoder attention backward (attn_bwd2) without its global loads
#     d6  attn_bwd2 without its compute loop
#     d7  LayerNorm backward path h using the bf16 values as x-hat directly (no affine inverse)
set -e
NAME=$1; REV=${2:-HEAD}
R=$(git rev-parse --show-toplevel); cd $R
D=_abc/$NAME; rm -rf $D; mkdir -p $D
git archive "$REV" jumbo_mae_tpu_amd tools bench.py | tar -x -C $D
python - $D/jumbo_mae_tpu_amd/csrc $NAME <<'PY'
import sys
csrc, name = sys.argv[1], sys.argv[2]

def edit(fname, start, end, reps):
    p = f"{csrc}/{fname}"
    s = open(p).read()
    a = s.index(start)
    b = s.index(end, a)
    body = s[a:b]
    for old, new in reps:
        assert old in body, old
        body = body.replace(old, new)
    open(p, "w").write(s[:a] + body + s[b:])

LOADS3 = """    if (i < SP * NCH && r < S) {
      qv[it] = *reinterpret_cast<const uint4*>(Qg + r * ts + c);
      kv[it] = *reinterpret_cast<const uint4*>(Kg + r * ts + c);
      dv[it] = *reinterpret_cast<const uint4*>(dOg + r * os + c);
      ov[it] = *reinterpret_cast<const uint4*>(Og + r * os + c);
    }"""
VLOAD3 = "if (key < S) vf[w][kk] = ld8(Vg + (long)key * ts + 32 * kk + 8 * g);"
B3 = ("void attn_bwd3_kernel(", "// forward images: row-major K and V")
B2 = ("void attn_bwd2_kernel(", "// attn_bwd2_kernel's layout with the per-key-tile work batched")
if name == "d1":
    edit("attention.hip", *B3, [(VLOAD3, ""), (LOADS3, LOADS3.replace("r < S) {", "r < S && S < 0) {", 1))])
elif name == "d2":
    edit("attention.hip", *B3, [("for (int qc = 0; qc * QC < SP; ++qc) {", "for (int qc = 0; qc * QC < SP && S < 0; ++qc) {")])
elif name == "d3":
    edit("attention.hip", *B3, [(LOADS3, """    if (i < SP * NCH && r < S) {
      kv[it] = *reinterpret_cast<const uint4*>(Kg + r * ts + c);
    }""")])
elif name == "d4":
    edit("attention.hip", *B3, [(VLOAD3, ""), (LOADS3, """    if (i < SP * NCH && r < S) {
      qv[it] = *reinterpret_cast<const uint4*>(Qg + r * ts + c);
      dv[it] = *reinterpret_cast<const uint4*>(dOg + r * os + c);
      ov[it] = *reinterpret_cast<const uint4*>(Og + r * os + c);
    }""")])
elif name == "d5":
    edit("attention.hip", *B2, [("  auto load_regs = [&](int b) {\n", "  auto load_regs = [&](int b) {\n    if (S > 0) { lsen = 0.f; return; }\n")])
elif name == "d6":
    edit("attention.hip", *B2, [("  for (int qc = 0; qc * QC < SP; ++qc) {\n    // one key tile;",
                                 "  for (int qc = 0; qc * QC < SP && S < 0; ++qc) {\n    // one key tile;")])
elif name == "d7":
    edit("layernorm.hip", "void ln_bwd_kernel(", "// out_k[c] += sum_b ws", [("""          if constexpr (HP) {  // x-hat = (h - beta) / gamma
            float bb[4], ig[4];
            load4(hbi + col, bb);
            load4(hbi + D + col, ig);
#pragma unroll
            for (int j = 0; j < 4; ++j) xh[i][j] = (xh[i][j] - bb[j]) * ig[j];
          } else {""", """          if constexpr (HP) {  // DIAGNOSTIC: bf16 x-hat read as is (no transform)
          } else {""")])
else:
    raise SystemExit(f"unknown diagnostic {name}")
PY
(cd $D && python -m jumbo_mae_tpu_amd.csrc.build --variant release > /dev/null)
rm -rf $D/build
ls $D/jumbo_mae_tpu_amd/_C*.so
