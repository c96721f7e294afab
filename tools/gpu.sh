#!/bin/bash
# Rebuild libensvs.so, verify the C ABI binding, then run a command on the MI355X box.
# usage: tools/gpu.sh <timeout-seconds> '<command>'
set -e
cd "$(dirname "$0")/.."
make -j8 >/dev/null
python -m pytest tests/test_capi.py -q >/dev/null
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
