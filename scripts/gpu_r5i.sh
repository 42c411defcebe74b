#!/bin/bash
# round-5 session I: unit profiles (trace, FETCH / WRITE, SQ) of the weighted
# F100k sweep (seeds' Dial + rows) and of the M1M part
set -u
PROF_ARGS="--topology fabric100k-w" bash scripts/gpu_r5e.sh ${1:-i1}w || exit 1
PROF_ARGS="--topology mesh1m --part-of 122" bash scripts/gpu_r5e.sh ${1:-i1}m
