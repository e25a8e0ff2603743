#!/bin/bash
./gpu_cmd.sh || exit $?
./gpu_prof.sh ${1:-r01}
