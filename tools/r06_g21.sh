# round 6: caller split-K on the split-role rings for the long-K N = 768 products (A/B)
set -o pipefail
O=gpurun_out/g21; mkdir -p $O
timeout -k 10 300 python -u tools/ab/roles_split_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cut -c1-110 $O/ab.txt
