#!/bin/bash
# Same-box A/B of the NAT established-flow leg: the dnat GPU tests with the
# product library, then `bench.py --only dnat --lib L` twice per library
# (interleaved). Libraries named below are built by hand (make OUT=...).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dnat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dnat.log 2>&1 || exit 5
for r in 1 2; do for L in abl/libwm_old.so abl/libnat_occ8.so; do
  timeout -k 10 200 python bench.py --only dnat --no-cpu --lib $L > gpurun_out/nat_$(basename $L .so)_$r.json 2>> gpurun_out/nat.err || exit 6
done; done
