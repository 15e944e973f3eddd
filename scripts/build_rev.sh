#!/bin/bash
# Build the engine library of git revision REV as the experiment library
# custom_envs_amd/lib/libcustom_envs_amd_NAME.so (CE_LIB=NAME selects it),
# for interleaved A/B runs of the current tree against an earlier one.
#   scripts/build_rev.sh REV NAME [DEFINE...]
set -eu
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" worktree add -q --detach "$TMP" "$REV"
trap 'git -C "$ROOT" worktree remove --force "$TMP"' EXIT
( cd "$TMP" && python -c "
import sys; sys.path.insert(0, '.')
from custom_envs_amd import build
print(build.build(variant='$NAME', defines=sys.argv[1:]))" "$@" )
cp "$TMP/custom_envs_amd/lib/libcustom_envs_amd_$NAME.so" "$ROOT/custom_envs_amd/lib/"
echo "built custom_envs_amd/lib/libcustom_envs_amd_$NAME.so from $REV"
