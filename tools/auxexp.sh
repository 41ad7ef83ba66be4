for aux in 0 1 2 3 4; do
  PQG_GATHER_AUX=$aux BWS="12 16 20" bash tools/bw_sweep.sh aux$aux || exit 1
done
