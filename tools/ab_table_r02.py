import json,glob,collections,sys
res=collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob('gpurun_out/ab_*_*.log')):
    name=f.split('/')[-1][3:-4]
    v,rest=name.split('_',1)
    cfg=rest.rsplit('_',1)[0]
    try: d=json.loads([l for l in open(f) if l.startswith('{')][0])
    except Exception as e: continue
    if cfg=='headline': x=(d['value'], d['kernels']['encode']['frac'], d['kernels']['decode_1erasure']['frac'])
    elif cfg=='mixed': x=(d['value'],)+tuple(round(c['encode_frac'],3) for c in d['classes'].values())+tuple(round(c['decode_frac'],3) for c in d['classes'].values())
    elif cfg=='rs12': x=(d['value'], d['kernels']['decode_2erasure']['frac'], d['kernels']['encode']['frac'])
    elif cfg.startswith('flows'): x=(d['value'],)+tuple(k['frac'] for k in d['kernels'].values())
    else: x=(d['value'], d['roofline']['frac'])
    res[cfg][v].append(x)
for cfg in res:
    print(cfg)
    for v in sorted(res[cfg]): print('  ',v, res[cfg][v])
