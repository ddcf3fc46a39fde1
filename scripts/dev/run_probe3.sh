set -u
O=gpurun_out/probe3; mkdir -p $O
CPK_LIB=capnp-zig_amd/lib/cap16k.so timeout -k 10 240 bash scripts/dev/c5_timeline.sh probe3/cap > /dev/null 2>&1 || exit $?
CPK_LIB=capnp-zig_amd/lib/e4.so timeout -k 10 240 bash scripts/dev/c5_timeline.sh probe3/base > /dev/null 2>&1 || exit $?
echo BASE; tail -20 $O/base/timeline.txt; echo CAP; tail -20 $O/cap/timeline.txt
