set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 200 python scripts/load_order_probe.py || exit $?
  timeout -k 10 200 python scripts/load_order_probe.py --first libflsgpu_exp.so || exit $?
  timeout -k 10 200 python scripts/load_order_probe.py --first libflsgpu_same.so || exit $?
done
