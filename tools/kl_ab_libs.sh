set -e
for lib in $LIBS; do
  echo "== $lib"; GTF_LIB=$PWD/gnn-track-finding_amd/gtf/$lib timeout -k 10 200 python -u tools/kl_ab.py 2>&1 | grep "ordered=1" | head -2
done
