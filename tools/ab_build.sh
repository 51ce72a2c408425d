#!/bin/bash
# Build the extension from git revision REV's csrc/ (everything else from the working tree)
# into ab/A_C.so and the working tree's into ab/B_C.so, for same-box A/B timing:
#   CSED_NATIVE_SO=$PWD/ab/A_C.so python bench.py ...   vs   CSED_NATIVE_SO=$PWD/ab/B_C.so ...
# usage: tools/ab_build.sh REV
set -e
REV=${1:?git revision}
cd "$(dirname "$0")/.."
mkdir -p ab
rm -rf /tmp/ab_csrc && cp -r csrc /tmp/ab_csrc
trap 'rm -rf csrc && cp -r /tmp/ab_csrc csrc' EXIT
git archive "$REV" csrc | tar -x -C /tmp/ab_rev_unpack 2>/dev/null || { mkdir -p /tmp/ab_rev_unpack && git archive "$REV" csrc | tar -x -C /tmp/ab_rev_unpack; }
rm -rf csrc && cp -r /tmp/ab_rev_unpack/csrc csrc && rm -rf /tmp/ab_rev_unpack
python -c "import __graft_entry__ as g; g.build()" > /dev/null
cp csed_514_project_distributed_training_using_pytorch_amd/_C.so ab/A_C.so
rm -rf csrc && cp -r /tmp/ab_csrc csrc
trap - EXIT
python -c "import __graft_entry__ as g; g.build()" > /dev/null
cp csed_514_project_distributed_training_using_pytorch_amd/_C.so ab/B_C.so
echo "ab/A_C.so = $REV, ab/B_C.so = working tree"
