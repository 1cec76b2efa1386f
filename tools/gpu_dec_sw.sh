#!/bin/bash
# Decoder tests + model parity, then the sliding-window bench and its kernel profile.
set -o pipefail
TAG=${1:-ds}
tools/gpu_dec.sh ${TAG} || exit $?
tools/gpu_swprof.sh ${TAG}
