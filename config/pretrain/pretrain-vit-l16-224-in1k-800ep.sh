#!/usr/bin/env bash
# ViT-L/16 Jumbo MAE pretraining, ImageNet-1k, 800 epochs, global batch 4096.
source "$(dirname "$0")/../_launch.sh"
BS=4096; N=1281167
launch main_pretrain.py --mode pretrain --image_mask_ratio 0.75 \
  --output-dir "$CKPT_DIR" --train-dataset-shards "$TRAIN_SHARDS" --valid-dataset-shards "$VALID_SHARDS" \
  --train-batch-size $BS --valid-batch-size 512 --train-loader-workers 40 --valid-loader-workers 10 \
  --random-crop rrc --color-jitter 0.0 --auto-augment none --random-erasing 0.0 --augment-repeats 1 \
  --test-crop-ratio 0.875 --mixup 0.0 --cutmix 0.0 \
  --layers 24 --dim 1024 --heads 16 --labels 0 --patch-size 16 --image-size 224 \
  --posemb sincos2d --pooling cls --dropout 0.0 --droppath 0.0 \
  --dec-layers 8 --dec-dim 512 --dec-heads 16 --dec-posemb sincos2d --dec-dropout 0.0 --dec-droppath 0.0 \
  --init-seed 0 --mixup-seed 0 --dropout-seed 0 --noise-seed 0 --shuffle-seed 0 \
  --optimizer adamw --learning-rate 1.5e-4 --weight-decay 0.05 --adam-b1 0.9 --adam-b2 0.95 --adam-eps 1e-8 \
  --lr-decay 1.0 --clip-grad 0.0 --grad-accum 1 \
  --warmup-steps $((N * 40 / BS)) --training-steps $((N * 800 / BS)) \
  --log-interval 1000 --eval-interval $((N / BS)) \
  --project MAE-JAX --name "$(basename "$0" .sh)" "$@"
