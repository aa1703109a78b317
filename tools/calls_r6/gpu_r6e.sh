#!/bin/bash
# After the readlane sign fix: lane / rx-batch / session / C++ API tests, the
# wrap job on the library without the poisoning (expected to fail), per-call
# echo; then fan-out A/B of fewer waves per message (more key registers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r6e tools/calls_r6/gpu_r6a.sh && TAG=r6e_fan VARIANTS="${VARIANTS:-base aux17 kv4w4 kv8w2 kv8w3 kv8w2a17 kv4w4c3 kv8w2c8}" tools/calls_r6/gpu_r6b.sh
