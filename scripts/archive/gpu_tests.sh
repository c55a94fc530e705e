#!/bin/bash
source "$(dirname "$0")/gpu_round.sh"
run gputests 1200 python -m pytest tests -q -m gpu
