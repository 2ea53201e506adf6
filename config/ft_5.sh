#!/usr/bin/env bash
# ft.sh sweep point: learning rate 6.0e-4, color jitter 0.3.
LR=6.0e-4 COLOR_JITTER=0.3 NAME=ft_5 exec "$(dirname "$0")/ft.sh" "$@"
