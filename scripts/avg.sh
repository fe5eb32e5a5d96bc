#!/bin/bash
# avg.sh [pattern] — mean / min / max of the "<label> : <value>" numbers that
# match `pattern` (default "gather") in every out-*.txt of the current
# directory (the TIME lines of mpi_daxpy_nvtx_*).  Reference: /root/reference/avg.sh.
pat=${1:-gather}
echo "PATTERN=$pat"
for f in *.txt; do
  [ -e "$f" ] || continue
  grep -v "^#" "$f" | grep -- "$pat" | awk -F: -v file="$f" '
    { v = $NF + 0; s += v; n += 1; if (n == 1 || v < lo) lo = v; if (n == 1 || v > hi) hi = v }
    END { if (n) printf "%s mean=%g min=%g max=%g n=%d\n", file, s / n, lo, hi, n }'
done
