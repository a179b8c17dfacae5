cd $GRAFT_REPO_ROOT
for pc in 8192 65536 512; do
  echo "== HSA_ANY_PCAP=$pc"
  HSA_ANY_PCAP=$pc timeout -k 10 100 python -u tools/exp/diag_anyq2.py > gpurun_out/dq_$pc.log 2>&1 || exit 1
  grep -E "^read |differing" gpurun_out/dq_$pc.log | head -8
done
