#!/bin/bash
# round 5 job 48: the round-end check on the current tree (GPU tests, smoke, the four recipe benches)
scripts/round_check.sh || exit $?
