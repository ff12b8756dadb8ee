#!/bin/bash
# Build rlcard_amd/libcardsim_<name>.so from the csrc/ of a git revision (default HEAD), for A/B runs against the
# working tree:  bash tools/build_head_variant.sh <name> [rev]
set -e
NAME=$1; REV=${2:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/csrc_XXXX)
mkdir -p $T/rlcard_amd/csrc $T/include
git -C $R archive $REV rlcard_amd/csrc include | tar -x -C $T
make -s -C $T/rlcard_amd/csrc OUT=$R/rlcard_amd/libcardsim_$NAME.so
rm -rf $T
echo built $R/rlcard_amd/libcardsim_$NAME.so from $REV
