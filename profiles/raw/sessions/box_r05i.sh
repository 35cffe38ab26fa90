#!/bin/bash
# Round-5 box session I: are a burst's slow first API answers its API server's cores waking up?
# Interleaved headline runs, API server IO threads sleeping (default) vs polling 5 ms after
# their last event, with the bind hops by tenth of the burst. usage: tools/box_r05i.sh OUT
set -o pipefail
OUT="$1" REPS=3 tools/box_decile_ab.sh "" "--apiserver-spin-us 5000"
