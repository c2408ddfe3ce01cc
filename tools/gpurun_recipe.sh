#!/bin/bash
# Local wrapper: stamp the tree's HEAD (plus "+dirty" when sources differ) into .git_head,
# then run one tools/gpu.sh recipe on a GPU box through gpurun.
#   tools/gpurun_recipe.sh <timeout-s> <recipe> <tag> [args]
t=$1; shift
cd "$(dirname "$0")/.." || exit 1
h=$(git rev-parse --short HEAD)
git diff --quiet HEAD -- . ':(exclude)profiles' || h="$h+dirty"
echo "$h" > .git_head
exec /usr/local/graft/bin/gpurun --timeout "$t" -- "bash tools/gpu.sh $*"
