#!/usr/bin/env bash
# Host-side helper: freeze the working tree into .snap/ (sent to the GPU box with the
# rest of the repo) so a queued gpurun call runs exactly this state even if the tree
# is edited while the call waits for a box. GPU scripts run from .snap and write
# their results to $GRAFT_REPO_ROOT/gpurun_out/.
set -e
cd "$(dirname "$0")/.."
rm -rf .snap
mkdir .snap
tar --exclude ./.snap --exclude ./.git --exclude ./gpurun_out --exclude ./build --exclude ./profiles \
    --exclude '__pycache__' --exclude ./.hypothesis --exclude '*.log' --exclude ./.pytest_cache -cf - . | tar -xf - -C .snap
echo "snapshot: $(du -sh .snap | cut -f1)"
