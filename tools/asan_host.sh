#!/bin/bash
# Host-only sanitizer runs (no GPU code is instrumented -- GPU sanitizers are not available on the
# pool): libecamd_host.so and liberasurecode.so.1 rebuilt with -fsanitize=address,undefined into
# /tmp/ecamd-asan, and the CPU tests that drive them run against those builds.
set -eo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O=/tmp/ecamd-asan
mkdir -p "$O"
cd "$R/liberasurecode_amd/csrc"
SAN="-O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -std=c++17 -I../../include -Ihost -Ihip"
g++ $SAN -shared -o "$O/libecamd_host.so" host/gf16.cpp host/tables.cpp host/xor_plan.cpp host/crc.cpp \
    host/bitslice.cpp host/host_api.cpp
g++ $SAN -DLIBERASURECODE_SO_SUFFIX='""' -shared -o "$O/liberasurecode.so.1" abi/frontend.cpp \
    -Wl,-soname,liberasurecode.so.1 -L../lib -l:libXorcode.so.1 -lz -ldl -lpthread \
    -Wl,--version-script=abi/frontend.map
cd "$R"
export ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export LD_LIBRARY_PATH="$R/liberasurecode_amd/lib"
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
python3 - <<PY
import sys
sys.path[:0] = ["$R", "$R/tests"]
from liberasurecode_amd import _lib
import ec_api
_lib.LIBDIR = "$O"
ec_api.LIB = "$O/liberasurecode.so.1"
import pytest
sys.exit(pytest.main(["-q", "-p", "no:cacheprovider", "tests/test_bitslice_host.py", "tests/test_host_planning.py",
                      "tests/test_percall_devices.py", "tests/test_frontend_cpu.py"]))
PY
