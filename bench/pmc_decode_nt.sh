R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_nt -o pmc -- python3 $R/bench/decode_cold.py --depth 2 14 --splits 1 --iters 20 > $R/gpurun_out/pmc_nt.log 2>&1
echo "rc=$?"
