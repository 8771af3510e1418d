ROUNDS=1 bash tools/ab_lib.sh libdmx.so libg4.so libg1.so
python -c "
import json
for l in ('libdmx','libg4','libg1'):
    for r in json.load(open('gpurun_out/bd_%s.json' % l))['records']:
        if r['layer']=='embed': print(l, round(r['ms']*1000,1))
"
