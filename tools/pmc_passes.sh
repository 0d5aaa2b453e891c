set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc -o fetch -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc -o write -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $R/gpurun_out/pmc -o req -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc_req.log 2>&1
