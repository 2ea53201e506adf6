#!/usr/bin/env bash
# Linear probe (frozen encoder, SyncBatchNorm + Dense head), LARS, batch 16384, 90 epochs.
source "$(dirname "$0")/../_launch.sh"
BS=${BS:-16384}; N=1281167
launch main_finetune.py --mode linear --output-dir "$CKPT_DIR" --pretrained-ckpt "$PRETRAINED" \
  --train-dataset-shards "$TRAIN_SHARDS" --valid-dataset-shards "$VALID_SHARDS" \
  --train-batch-size $BS --valid-batch-size 512 --train-loader-workers 40 --valid-loader-workers 10 \
  --random-crop rrc --color-jitter 0.0 --auto-augment none --random-erasing 0.0 --augment-repeats 1 \
  --test-crop-ratio 0.875 --mixup 0.0 --cutmix 0.0 --criterion ce --label-smoothing 0.0 \
  ${MODEL_FLAGS:---layers 12 --dim 768 --heads 12} --labels 1000 --patch-size 16 --image-size 224 \
  --posemb sincos2d --pooling cls --dropout 0.0 --droppath 0.0 \
  --init-seed 1 --mixup-seed 1 --dropout-seed 1 --shuffle-seed 1 \
  --optimizer ${OPT:-lars} --learning-rate ${LR:-0.1} --lr-decay 1.0 --clip-grad 0.0 --grad-accum 1 \
  --warmup-steps $((N * ${WARMUP_EP:-10} / BS)) --training-steps $((N * 90 / BS)) \
  --log-interval 10 --eval-interval $((N / BS)) \
  --project MAE-JAX --name "${NAME:-$(basename "$0" .sh)}" "$@"
