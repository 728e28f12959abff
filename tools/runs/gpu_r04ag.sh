# final round-4 build: the certificate at scale (default vs reference-order kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in "C3_ntru512 16777216" "C4_qary1024 4194304" "C5_ntru2048 262144"; do
  set -- $c
  echo "== cert $1 $2" && timeout -k 10 400 python -u tools/cert_mismatch.py --config $1 --total $2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-400 || exit 1
done
