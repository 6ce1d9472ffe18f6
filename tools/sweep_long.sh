set -o pipefail
for spec in "1200 o:10,2,2 10,2,3 10,2,2" "2000 o:8,4,3 8,4,3 8,4,2" "2500 o:8,8,3 10,4,3 10,4,2" "3000 o:8,8,3 6,8,2 6,8,3" "4000 o:8,8,3 8,8,2"; do
  set -- $spec; L=$1; shift
  echo "== len $L"
  timeout -k 10 200 python3 tools/sweep_variants.py --rounds 2 --len $L --batch 8192 --nseq 8000 "$@" 2>/dev/null | grep -h "GCUPS\|identical" || exit 1
done
