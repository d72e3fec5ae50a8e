#!/bin/bash
# Round 4: step timelines at HEAD (kernel trace, tools/gpu_timeline.sh) of the native 36^2x128 and the
# 196^2x198 U-Net steps, for the round-5 latency plan.
set -o pipefail
bash tools/gpu_timeline.sh unet1lip 128 36 12 && bash tools/gpu_timeline.sh unet1lip 198 196 12
