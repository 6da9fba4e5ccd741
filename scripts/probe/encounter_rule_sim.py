"""Candidate encounter rules replayed on scripts/probe/encounter_rule_study.py's per-level closest
approaches (profiles/r06c_encounter_rule_study.jsonl): for each rule, the proposals it would still end
ENCOUNTER where IAS15 integrates (2/0), the ones it would integrate where IAS15 raises (0/2), and how
many walkers it sends to which halving pass.  CPU only; run from the repository root."""
import itertools
import json

data = {}
for line in open("profiles/r06c_encounter_rule_study.jsonl"):
    d = json.loads(line)
    data[d["system"]] = d
def decide(r,kappa,sigma,maxp=3):
    for p,key in enumerate(("lv0","lv1","lv2","lv3")):
        v=r[key]; f=[x<1.0 for x in v]
        if not any(f): return p, False
        if all(f) and (max(v)<kappa or max(v)/min(v)-1<=sigma): return p, True
        if p==maxp: return p, all(f)
    return 3, None
for kappa,sigma in itertools.product([0.3,0.4,0.5],[0.02,0.05,0.1]):
    out=[]
    for s,d in data.items():
        e20=o02=0; st=[0,0,0,0]
        for r in d['rows']:
            p,enc=decide(r,kappa,sigma)
            st[p]+=1
            if r['ias15']==0 and enc: e20+=1
            if r['ias15']==2 and not enc: o02+=1
        out.append('%s:2/0=%d 0/2=%d stages=%s'%(s[:3],e20,o02,st))
    print(kappa,sigma,' | '.join(out))
print('--- two-stage rules (pass 1 is the last one an encounter can ask for)')
def decide2(r, at_p1, kappa=0.0, sigma=-1):
    v=r['lv0']; f=[x<1 for x in v]
    if not any(f): return 0, False
    if all(f) and (max(v)<kappa or max(v)/min(v)-1<=sigma): return 0, True
    if all(f) and sigma<0: return 0, True
    v=r['lv1']; f=[x<1 for x in v]
    if all(f): return 1, True
    if not any(f): return 1, False
    return 1, at_p1(v)
for name,fn in [('finest',lambda v:v[-1]<1),('two finest',lambda v:v[-1]<1 and v[-2]<1),('none',lambda v:False),('majority',lambda v:sum(x<1 for x in v)>=3)]:
  for kappa,sigma in [(0,-1),(0.4,0.05),(0.5,0.1),(0.6,0.1),(0.3,0.05)]:
    out=[]
    for s,d in data.items():
        e20=o02=0; st=[0,0]
        for r in d['rows']:
            p,enc=decide2(r,fn,kappa,sigma)
            st[p]+=1
            if r['ias15']==0 and enc: e20+=1
            if r['ias15']==2 and not enc: o02+=1
        out.append('%s:2/0=%d 0/2=%d p1=%d'%(s[:3],e20,o02,st[1]))
    print('%-10s k=%.1f s=%.2f'%(name,kappa,sigma),' | '.join(out))
print('--- rule A variants over the currently-ENC walkers')
rules={
 'A: unanimous main | p1 finest': lambda r: all(x<1 for x in r['lv0']) or r['lv1'][-1]<1,
 'A2: unanimous main | p1 two finest': lambda r: all(x<1 for x in r['lv0']) or (r['lv1'][-1]<1 and r['lv1'][-2]<1),
 'A3: unanimous main | p1 unanimous': lambda r: all(x<1 for x in r['lv0']) or all(x<1 for x in r['lv1']),
 'B: main finest | p1 finest (today w/o coarse-in-halving)': lambda r: r['lv0'][-1]<1 or r['lv1'][-1]<1,
 'C: unanimous main+ext | p1 finest': lambda r: (all(x<1 for x in r['lv0']) and r['ext']<1) or r['lv1'][-1]<1,
}
for name,fn in rules.items():
    out=[]
    for s,d in data.items():
        e20=sum(1 for r in d['rows'] if r['ias15']==0 and fn(r))
        o02=sum(1 for r in d['rows'] if r['ias15']==2 and not fn(r))
        p1=sum(1 for r in d['rows'] if not all(x<1 for x in r['lv0']))
        out.append('%s:2/0=%d 0/2=%d (of %d) newp1<=%d'%(s[:3],e20,o02,len(d['rows']),p1))
    print('%-45s'%name,' | '.join(out))
