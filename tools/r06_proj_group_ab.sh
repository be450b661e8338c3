set -euo pipefail
out=gpurun_out/r06p2; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in main pg2; do
    envs=""; [ $v = pg2 ] && envs="IMPLISOLID_PROJ_GROUP=2"
    for R in 128 256; do
      env $envs timeout -k 10 240 python3 tools/ob02_r512_probe.py 9 --baked --R $R > $out/${v}_${R}_$rep.log 2>&1
      echo "$v $rep $(grep config4s $out/${v}_${R}_$rep.log)" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
