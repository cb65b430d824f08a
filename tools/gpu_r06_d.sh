# Round 6, call D: where the N = 50 dual path's non-finite end-point multipliers
# come from (diagnostic build counters by re-solve path), modes 2 and 3
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python tools/diag_phases.py 20000 50 2 5 5 > $O/phases_n50m2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/diag_phases.py 20000 50 3 5 5 > $O/phases_n50m3.txt 2>&1 || exit $?
grep -h "non-finite\|handed to GI\|GI solves" $O/phases_n50m2.txt $O/phases_n50m3.txt
