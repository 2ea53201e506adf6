#!/usr/bin/env bash
# Linear probe ViT-L/16, LARS, batch 16384, 90 epochs.
MODEL_FLAGS="--layers 24 --dim 1024 --heads 16" NAME="$(basename "$0" .sh)" \
  exec "$(dirname "$0")/ln-lars-vit-b16-224-in1k.sh" "$@"
