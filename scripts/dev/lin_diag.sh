# Dev aid: linearisation kernel time of diagnostic variants (1: no matrix stores, 2: no model)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for v in product lin1 lin2; do
  if [ $v = product ]; then L=""; else L=build/variants/$v/libsrbd_qp.so; fi
  SRBD_QP_LIB=$L timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$v -o run -- python3 scripts/dev/lin_ls_prof.py none > /dev/null 2>&1 || exit 1
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/prof_$v/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
  if 'lin_' in x['Name']: print('$v', x['Name'][:50], '%.3f ms'%(float(x['AverageNs'])/1e6))
"
done
