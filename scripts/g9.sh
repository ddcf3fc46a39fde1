set -u
export TMPDIR=/tmp
for t in 128 26 230; do
CPK_LIB=capnp-zig_amd/lib_exp/prof.so timeout -k 10 120 python3 scripts/fill_prof.py $t 2>&1 | grep -v amdgpu.ids || exit 1
done
