export TMPDIR=/tmp; mkdir -p gpurun_out
PYTHONPATH=cuda-grmonty_amd python -c "from grmonty_amd.synth_dump import ensure_dump; ensure_dump('gpurun_out/synth192.dump', 192, 192)" || exit 1
for cfg in ${CFGS:-"product|" "product|29=0" "vhead|" "product|"}; do
  lib=${cfg%%|*}; o=${cfg#*|}
  L=""; [ $lib = product ] || L="cuda-grmonty_amd/ab/libgrmonty_amd_$lib.so"
  GRMONTY_AMD_LIB=$L OPTS="$o" EARLY=0 timeout -k 10 120 python -u tools/long_photon_bench.py 3 > gpurun_out/chx_$lib.log 2>&1 || { echo "fail $lib"; tail -3 gpurun_out/chx_$lib.log; exit 1; }
  echo "== $lib $o"; tail -3 gpurun_out/chx_$lib.log | cut -c1-200
done
rm -f gpurun_out/*.dump
