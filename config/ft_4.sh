#!/usr/bin/env bash
# ft.sh sweep point: learning rate 6.0e-4, color jitter 0.0.
LR=6.0e-4 COLOR_JITTER=0.0 NAME=ft_4 exec "$(dirname "$0")/ft.sh" "$@"
