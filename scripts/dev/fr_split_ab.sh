set -o pipefail
mkdir -p gpurun_out/frab
for i in 1 2; do
  timeout -k 10 200 env CPK_LIB=capnp-zig_amd/lib_exp/fr_old.so python3 bench.py --only rpc_framer_split > gpurun_out/frab/old$i.json 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --only rpc_framer_split > gpurun_out/frab/new$i.json 2>&1 || exit 1
done
