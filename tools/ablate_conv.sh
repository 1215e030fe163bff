cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in libnps_hip libnps_abl_PRODUCER libnps_abl_CONSUMER; do
  echo "== $L"
  NPS_HIP_LIB=$PWD/neural-pde-surrogates_amd/nps_hip/$L.so timeout -k 10 120 python3 tools/conv_bench.py --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 0 2>&1 | grep conv
  NPS_HIP_LIB=$PWD/neural-pde-surrogates_amd/nps_hip/$L.so timeout -k 10 120 python3 tools/conv_bench.py --cin 388 --cout 192 --k 1 --hw 260 --b 16 --gn 0 2>&1 | grep conv
done
