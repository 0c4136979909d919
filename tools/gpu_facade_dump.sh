set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fd
timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0,'tests')
import facade_build as fb, tempfile
d=tempfile.mkdtemp(); fb.write_states(d)
for sc in ['gradient','golden']:
    json.dump(fb.run('gpu', sc, d), open('gpurun_out/fd/gpu_'+sc+'.json','w'))
print('ok')
"
