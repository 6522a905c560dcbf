mkdir -p gpurun_out/lnab
for i in 1 2; do
for cap in 256 1024; do
  echo "cap $cap rep $i" >> gpurun_out/lnab/ab.txt
  ICAP_LN_BWD_PCAP=$cap ROWS=3200,3584 CASES=mapper,GPT-2 timeout -k 10 120 python -u tools/ab/ln_scale_probe.py >> gpurun_out/lnab/ab.txt 2>&1 || exit 1
done; done
cat gpurun_out/lnab/ab.txt | grep -v amdgpu.ids
