set -u
export PASSES="SQC_ICACHE_HITS;SQC_ICACHE_MISSES;SQC_ICACHE_MISSES_DUPLICATE;SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES"
for w in chain_65536 chain chorus; do
  timeout -k 10 400 bash tools/pmc_profile.sh "$w" 10 || exit $?
done
echo done
