# same-box timing of the product small-O rho-forward kernel against the probe's copy of the
# previous version (tools/xcws_probe.hip), at the C2 shapes and a 12-round + tail grid
set -o pipefail
for shape in "34 20 146 216000" "33 20 147 216000" "34 20 128 200000" ; do
  echo "## $shape"; timeout -k 10 60 tools/bin/xcws_probe $shape 20 | grep -E "product|full \(DIAG" | tail -3 || exit 1
done
