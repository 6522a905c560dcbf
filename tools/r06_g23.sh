# round 6: the A/B table with the 256 x 256 8-phase form added
set -o pipefail
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 300 python -u tools/ab/roles_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-125 $O/ab.txt
