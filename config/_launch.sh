#!/usr/bin/env bash
# Shared launcher: one process per MI355X over RCCL/xGMI via torchrun.
#   NGPU (default: all visible GPUs), NNODES/NODE_RANK/MASTER_ADDR/MASTER_PORT for multi-node.
#   DATA_DIR: directory or URL holding imagenet-1k-wds shards (the reference's $GCS_DATASET_DIR:
#   a local path, gs://bucket/..., s3://..., http(s)://..., or a "pipe:<cmd> " prefix such as
#   "pipe:gsutil cat gs://bucket"), CKPT_DIR: output dir or URL (default $DATA_DIR/CKPT; for a
#   pipe: prefix, the URL that ends the prefix + /CKPT), PRETRAINED: checkpoint path or URL for
#   finetune / linear probe (the reference's $GCS_MODEL_PATH).
set -euo pipefail
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
NGPU="${NGPU:-$(python3 -c 'import torch; print(max(torch.cuda.device_count(), 1))')}"
DATA_DIR="${DATA_DIR:-${GCS_DATASET_DIR:-$REPO/data}}"
if [[ "$DATA_DIR" == pipe:* ]]; then
  # a pipe: prefix is a READ command; checkpoints go to the URL it reads from (its last word)
  CKPT_DIR="${CKPT_DIR:-${DATA_DIR##* }/CKPT}"
else
  CKPT_DIR="${CKPT_DIR:-$DATA_DIR/CKPT}"
fi
PRETRAINED="${PRETRAINED:-${GCS_MODEL_PATH:-}}"
TRAIN_SHARDS="${TRAIN_SHARDS:-$DATA_DIR/imagenet-1k-wds/imagenet1k-train-{0000..1023}.tar}"
VALID_SHARDS="${VALID_SHARDS:-$DATA_DIR/imagenet-1k-wds/imagenet1k-validation-{00..63}.tar}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
launch() {  # launch <entry.py> <flags...>   (JMAE_DRYRUN=1: print the argv instead of running)
  local entry="$1"; shift
  if [ "${JMAE_DRYRUN:-0}" = "1" ]; then printf '%s\n' "$entry" "$@"; return 0; fi
  exec python3 -m torch.distributed.run --nnodes "${NNODES:-1}" --node-rank "${NODE_RANK:-0}" \
    --nproc-per-node "$NGPU" --master-addr "${MASTER_ADDR:-127.0.0.1}" --master-port "${MASTER_PORT:-29500}" \
    "$REPO/src/$entry" "$@" --hostname "$(hostname)"
}
