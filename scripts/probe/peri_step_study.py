"""Steady-state study (CPU, oracle): would a base step scaled to the ensemble's shortest pericentre
passage (tau = min over planets of P (1 - e)^1.5; dt = dt0 * tau_ens / tau0, gridded) remove the
halving passes at the bench chain's iteration 2000?  Oracle adaptive restatement vs IAS15 on the
6144 slots of scripts/probe/slots_it2000.npz: max |dlogL|, stage histogram (0 plan step, 1
extension, 1 + r halvings), halving directions and the work relative to the plan's step.
Output: profiles/r03r_peri_step_study.jsonl.  Usage: python scripts/probe/peri_step_study.py"""
import sys, os, json, numpy as np
ROOT=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0]=[os.path.join(ROOT,d) for d in ('rvel-mcmc_amd','oracle','tests')]
import oracle as O
from conftest import S2_PLANETS
from rvmcmc import engine
from concurrent.futures import ThreadPoolExecutor
def par(fn,P,nt=8):
    idx=np.array_split(np.arange(len(P)),nt)
    with ThreadPoolExecutor(nt) as ex: parts=list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]
def tau(X):  # X [W][10] rows m,a,h,k,l per planet
    t=[]
    for p in range(2):
        m,a,h,k=X[:,5*p],X[:,5*p+1],X[:,5*p+2],X[:,5*p+3]
        P=2*np.pi*np.sqrt(a**3/(1+m)); e=np.hypot(h,k)
        t.append(P*(1-e)**1.5)
    return np.min(t,axis=0)
cfg=engine.IntegratorConfig()
x0=np.array([[p[k] for k in 'm a h k l'.split()] for p in S2_PLANETS]).reshape(1,-1)
dt0,mult,_=cfg.plan_args(S2_PLANETS); tol,rmax,g0,_=cfg.resolve(S2_PLANETS)
t0=tau(x0)[0]; D=dt0/t0
ens=np.load(os.path.join(ROOT,'profiles','r03_bench_ensemble.npz'))['it2000']
d=np.load(os.path.join(ROOT,'scripts','probe','slots_it2000.npz'))
obs=O.OracleObs(tf=d['tf'],tb=d['tb'],rvf=d['rvf'],rvb=d['rvb'],errorf=d['errorf'],errorb=d['errorb'],Npoints=100)
te=tau(ens); ts=tau(d['K'])
print('tau0',t0,'ens min',te.min(),'q01',np.quantile(te,.001),'slots min',ts.min())
X=d['K']; P=np.zeros((len(X),2,7)); P[:,:,:5]=X.reshape(-1,2,5)
li,si=par(lambda p:O.logl_ias15_batch(p,2,obs),P)
imin=np.argmin(te); w=ens[imin]
pl=[dict(m=w[5*p],a=w[5*p+1],h=w[5*p+2],k=w[5*p+3],l=w[5*p+4]) for p in range(2)]
for name,dt,g in [('plan0',dt0,g0)]+[(f'ens_min/{f}',D*te.min()/f,cfg.ecc_guard(pl)) for f in (1.0,1.2)]:
    dtg=2.0**(round(np.log2(dt)*16)/16)
    la,sa,rf,_,_=par(lambda p:O.logl_whx_adapt_batch(p,2,obs,dtg,mult,tol,rmax,ecc_guard=g),P)
    ok=(sa==0)&(si==0); e=np.abs(la-li)[ok]
    print(json.dumps(dict(name=name,dt=dtg,dt_ratio=dt0/dtg,guard=g,max=float(e.max()),n1e6=int((e>1e-6).sum()),hist=np.bincount(rf.ravel(),minlength=6).tolist(),halv=int((rf>=2).sum()),work=float((2.0**np.maximum(rf-1,0)).mean()*dt0/dtg))),flush=True)
