#!/bin/bash
# final rocprofv3 passes of this build, then the RNA path at C3 scale
bash tools/gpu/prof.sh r03 || exit $?
bash tools/gpu/r03t.sh
