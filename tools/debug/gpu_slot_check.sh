#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/tensorflow_distributed_amd
echo "== base"; timeout -k 10 200 python tools/debug/bn_slot_atomics.py && \
echo "== atomic wait"; TFD_NATIVE_LIB=$L/_C_aw.so timeout -k 10 200 python tools/debug/bn_slot_atomics.py && \
echo "== race base"; timeout -k 10 200 python tools/debug/bn_slot_race.py && \
echo "== race atomic wait"; TFD_NATIVE_LIB=$L/_C_aw.so timeout -k 10 200 python tools/debug/bn_slot_race.py
