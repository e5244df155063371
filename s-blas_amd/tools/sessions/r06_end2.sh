# r06 end set (2/2): FETCH / WRITE / L2 passes for the kernels configs[1] and
# configs[2] name (row split and CSR5 over their XCD panels, config 2) and for
# configs[3]'s SpMM C tile (bench.py's config4 leg alone).
set -o pipefail
O=gpurun_out/r06end; mkdir -p $O
export TMPDIR=/tmp
NOLEG="--steps 5 --warmup 1 --no-cpu-baseline --no-check --no-config3 --no-config4 --no-config5 --no-structured --no-rowsplit-beside --no-peak"
run3() {  # name, bench args
  for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:l2"; do
    C=${pass%%:*}; D=${pass##*:}
    timeout -s KILL 150 rocprofv3 --pmc $C -d $O/$1_$D -o run --output-format csv -- python3 bench.py $2 > $O/$1_$D.log 2>&1 || return 1
  done
}
run3 rs "--algo rowsplit $NOLEG" || exit 1
python3 s-blas_amd/tools/pmc_traffic.py --kernel "k_spmv_panel,k_panel_reduce" --fetch $O/rs_fetch --write $O/rs_write --l2 $O/rs_l2 --algorithmic 533000004 --out $O/pmc_rowsplit.json > /dev/null || exit 1
run3 c5 "--algo csr5 $NOLEG" || exit 1
python3 s-blas_amd/tools/pmc_traffic.py --kernel "k_spmv_csr5_panel,k_csr5_calibrate_panel,k_panel_reduce" --fetch $O/c5_fetch --write $O/c5_write --l2 $O/c5_l2 --algorithmic 533000004 --out $O/pmc_csr5.json > /dev/null || exit 1
SP="--steps 5 --warmup 1 --no-cpu-baseline --no-check --no-config3 --no-config5 --no-structured --no-rowsplit-beside --no-peak --nrows 20000"
run3 mm "$SP" || exit 1
python3 s-blas_amd/tools/pmc_traffic.py --kernel "k_spmm_ctile,k_spmm_ctreduce" --fetch $O/mm_fetch --write $O/mm_write --l2 $O/mm_l2 --algorithmic 699177252 --out $O/pmc_spmm_ctile.json > /dev/null
