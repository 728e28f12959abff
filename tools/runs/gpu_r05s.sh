# round 5 final build: the certificate at scale (default vs reference-order kernel:
# C3 2^24, C4 2^22, C5 2^18, every coefficient compared)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05s
: > gpurun_out/${TAG}_cert.log
for c in "C3_ntru512 16777216" "C4_qary1024 4194304" "C5_ntru2048 262144"; do set -- $c
  echo "== cert $1 $2" && timeout -k 10 400 python -u tools/cert_mismatch.py --config $1 --total $2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-400 | tee -a gpurun_out/${TAG}_cert.log || exit 1
done
