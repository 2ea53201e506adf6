#!/usr/bin/env bash
# ViT-B/16 end-to-end finetuning from a Jumbo-MAE checkpoint: 110 epochs, global batch 1024,
# AdamW + layer-wise LR decay, RandAugment, Mixup/CutMix, label smoothing, droppath.
# LR / COLOR_JITTER / WD / LR_DECAY / NAME may be overridden (ft_2..ft_5 and loop_* use them).
source "$(dirname "$0")/_launch.sh"
BS=1024; N=1281167
launch main_finetune.py --mode finetune --output-dir "$CKPT_DIR" --pretrained-ckpt "$PRETRAINED" \
  --train-dataset-shards "$TRAIN_SHARDS" --valid-dataset-shards "$VALID_SHARDS" \
  --train-batch-size $BS --valid-batch-size 512 --train-loader-workers 40 --valid-loader-workers 10 \
  --random-crop rrc --color-jitter "${COLOR_JITTER:-0.0}" --auto-augment "rand-m9-mstd0.5-inc1" \
  --random-erasing 0.0 --augment-repeats 1 --test-crop-ratio 0.875 --mixup 0.8 --cutmix 1.0 \
  --criterion ce --label-smoothing 0.1 \
  --layers 12 --dim 768 --heads 12 --labels 1000 --patch-size 16 --image-size 224 \
  --posemb sincos2d --pooling cls --dropout 0.0 --droppath 0.1 \
  --init-seed 1 --mixup-seed 1 --dropout-seed 1 --shuffle-seed 1 \
  --optimizer adamw --learning-rate "${LR:-3.0e-3}" --weight-decay "${WD:-0.05}" --lr-decay "${LR_DECAY:-0.75}" \
  --clip-grad 0.0 --grad-accum 1 \
  --warmup-steps $((N * 10 / BS)) --training-steps $((N * 110 / BS)) \
  --log-interval 10 --eval-interval $((N / BS)) \
  --project MAE-JAX --name "${NAME:-$(basename "$0" .sh)}" "$@"
