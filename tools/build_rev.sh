#!/bin/bash
# Build libppe_hip.so of git revision REV as packet-process-engine_amd/libppe_hip_NAME.so (for in-process A/B runs
# of one revision against another with tools/ab_bench.py).   usage: tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" include packet-process-engine_amd | tar -x -C "$T"
make -s -C "$T/packet-process-engine_amd" -j8 >/dev/null
cp "$T/packet-process-engine_amd/libppe_hip.so" "$ROOT/packet-process-engine_amd/libppe_hip_$NAME.so"
rm -rf "$T"
echo "built packet-process-engine_amd/libppe_hip_$NAME.so from $REV"
