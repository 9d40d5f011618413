import json,sys,glob,collections,statistics as st
d=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1]+'/*.jsonl'):
    parts=f.split('/')[-1][:-6].rsplit('_',2)
    if len(parts)!=3 or parts[1] not in ('reg','staged'): continue
    name,mode,r=parts
    for l in open(f):
        if l.startswith('{'):
            x=json.loads(l); assert x['verified']
            d[(mode,x['packets'])][name].append((x['encap_ms']*1e3,x['decap_ms']*1e3))
names=sys.argv[2].split(',')
for mode in ('reg','staged'):
    print(mode, ''.join(f'{n:>16}' for n in names))
    for p in sorted({k[1] for k in d}):
        row=d[(mode,p)]
        print(f'{p:6d}',''.join('%8.0f/%-7.0f'%(min(a for a,b in row[n]),min(b for a,b in row[n])) if row[n] else ' '*16 for n in names))
