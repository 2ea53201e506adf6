#!/usr/bin/env bash
# Finetune grid: weight decay {0.06, 0.07} x learning rate {1e-3, 3e-3}, layer decay 0.65.
for wd in 0.06 0.07; do
  for lr in 1e-3 3e-3; do
    echo "Running with weight_decay=${wd}, learning_rate=${lr}"
    WD=$wd LR=$lr LR_DECAY=0.65 NAME="loop_1_wd${wd}_lr${lr}" bash "$(dirname "$0")/ft.sh" "$@"
  done
done
