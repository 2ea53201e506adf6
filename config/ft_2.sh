#!/usr/bin/env bash
# ft.sh sweep point: learning rate 1.0e-3, color jitter 0.0.
LR=1.0e-3 COLOR_JITTER=0.0 NAME=ft_2 exec "$(dirname "$0")/ft.sh" "$@"
