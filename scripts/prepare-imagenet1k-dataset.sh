#!/usr/bin/env bash
# Fetch the webdataset-format ImageNet-1k shards (timm/imagenet-1k-wds on the HF hub) into
# $DATA_DIR/imagenet-1k-wds/ (1024 train + 64 validation tars). Needs HF_TOKEN and network.
set -euo pipefail
DATA_DIR="${DATA_DIR:-${GCS_DATASET_DIR:-./data}}"
OUT="$DATA_DIR/imagenet-1k-wds"
mkdir -p "$OUT"
BASE="https://huggingface.co/datasets/timm/imagenet-1k-wds/resolve/main"
fetch() { curl -fL -H "Authorization: Bearer ${HF_TOKEN:?set HF_TOKEN}" -o "$OUT/$1" "$BASE/$1"; }
for i in $(seq -f "%04g" 0 1023); do fetch "imagenet1k-train-$i.tar"; done
for i in $(seq -f "%02g" 0 63); do fetch "imagenet1k-validation-$i.tar"; done
echo "shards in $OUT"
