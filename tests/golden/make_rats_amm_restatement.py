"""Independent numpy restatement of the config-3 rats Gibbs+AMM scheme, written from
src/samplers/amm.jl:66-108 (sample!, setadapt!) and doc/examples/rats.jl:48-97, sharing no
code with oracle/oracle.c or the HIP kernels (numpy RNG, numpy's unpivoted Cholesky: the
pivot order changes the factor, not the proposal distribution).  It fixes what the
reference's own always-adapting AMM gives for s2_c over the rats.rst run length
(10000 iterations, burnin 2500), so the GPU's value can be checked against the reference
algorithm rather than against the long-run posterior it approaches slowly.

  python tests/golden/make_rats_amm_restatement.py K T B adapt|noadapt [out.json]
"""
import numpy as np, sys
y=np.array([151,199,246,283,320,145,199,249,293,354,147,214,263,312,328,155,200,237,272,297,135,188,230,280,323,159,210,252,298,331,141,189,231,275,305,159,201,248,297,338,177,236,285,350,376,134,182,220,260,296,160,208,261,313,352,143,188,220,273,314,154,200,244,289,325,171,221,270,326,358,163,216,242,281,312,160,207,248,288,324,142,187,234,280,316,156,203,243,283,317,157,212,259,307,336,152,203,246,286,321,154,205,253,298,334,139,190,225,267,302,146,191,229,272,302,157,211,250,285,323,132,185,237,286,331,160,207,257,303,345,169,216,261,295,333,157,205,248,289,316,137,180,219,258,291,153,200,244,286,324],float).reshape(30,5)
Xm=np.array([8,15,22,29,36.])-22
K=int(sys.argv[1]); T=int(sys.argv[2]); B=int(sys.argv[3]); mode=sys.argv[4]
rng=np.random.default_rng(5)
a=y.mean(1)+rng.normal(0,3,(K,30)); b=(y*Xm).sum(1)/490+rng.normal(0,.3,(K,30))
ma=np.where(np.arange(K)%2==0,150.,15.); mb=np.where(np.arange(K)%2==0,10.,1.)
sc=np.where(np.arange(K)%2==0,1.,10.); sa=sc.copy(); sb=sc.copy()
def ig(shape,scale): return scale/rng.gamma(shape,1.0,size=scale.shape)
n=30
class Tune: pass
def newtune(sig):
    t=Tune(); t.m=np.zeros(K,int); t.Mv=None; t.Mvv=None; t.Lm=np.zeros((K,n,n)); t.L=np.sqrt(sig)*np.eye(n); t.fresh=True; return t
ta=newtune(1.0); tb=newtune(0.01)
def lp_alpha(av):   # logpdf!(alpha block): prior + y
    r=y[None]-av[:,:,None]-b[:,:,None]*Xm
    return (-0.5*(av-ma[:,None])**2/sa[:,None]).sum(1) -0.5*(r**2).sum((1,2))/sc
def lp_beta(bv):
    r=y[None]-a[:,:,None]-bv[:,:,None]*Xm
    return (-0.5*(bv-mb[:,None])**2/sb[:,None]).sum(1) -0.5*(r**2).sum((1,2))/sc
def amm(v,t,lpf):
    if t.fresh:
        t.Mv=v.copy(); t.Mvv=v[:,:,None]*v[:,None,:]; t.fresh=False; alias=True
    else: alias=False
    x=rng.normal(size=(K,n))@t.L.T
    use=t.m>2*n
    z2=rng.normal(size=(K,n)); y2=np.einsum('kij,kj->ki',t.Lm,z2)
    if mode=='noadapt': use[:]=False
    x=np.where(use[:,None],0.05*x+0.95*y2,x)
    x=x+v
    acc=rng.random(K)<np.exp(lpf(x)-lpf(v))
    v=np.where(acc[:,None],x,v)
    if mode=='noadapt': return v
    t.m+=1; p=(t.m/(t.m+1.0))[:,None]
    if alias: t.Mv=v.copy()
    else: t.Mv=p*t.Mv+(1-p)*v
    t.Mvv=p[:,:,None]*t.Mvv+(1-p)[:,:,None]*v[:,:,None]*v[:,None,:]
    if t.m[0]>=n+2:
        S=(2.38**2/n/p[:,:,None])*(t.Mvv-t.Mv[:,:,None]*t.Mv[:,None,:])
        if mode=='sym': S=0.5*(S+S.transpose(0,2,1))
        try: t.Lm=np.linalg.cholesky(S)
        except np.linalg.LinAlgError:
            for k in range(K):
                try: t.Lm[k]=np.linalg.cholesky(S[k])
                except np.linalg.LinAlgError: pass
    return v
Sy=y.sum(1); Sxy=(y*Xm).sum(1)
acc=[]
for it in range(T):
    r=y[None]-a[:,:,None]-b[:,:,None]*Xm
    sc=ig(0.001+75,0.001+0.5*(r**2).sum((1,2)))
    a=amm(a,ta,lp_alpha)
    vv=1/(30/sa+1e-6); ma=vv*(a.sum(1)/sa)+np.sqrt(vv)*rng.normal(size=K)
    sa=ig(0.001+15,0.001+0.5*((a-ma[:,None])**2).sum(1))
    b=amm(b,tb,lp_beta)
    vv=1/(30/sb+1e-6); mb=vv*(b.sum(1)/sb)+np.sqrt(vv)*rng.normal(size=K)
    sb=ig(0.001+15,0.001+0.5*((b-mb[:,None])**2).sum(1))
    if it>=B: acc.append([sc.mean(),mb.mean(),(ma-22*mb).mean()])
acc=np.array(acc)
print(mode, acc.mean(0))
if len(sys.argv) > 5:
    import json
    json.dump({"chains": K, "iters": T, "burnin": B, "mode": mode, "scheme": "rats_scheme_gibbs_amm",
               "mean": dict(zip(["s2_c", "mu_beta", "alpha0"], acc.mean(0).tolist())),
               "note": "per-iteration chain averages over the kept window; numpy PCG64 seed 5"},
              open(sys.argv[5], "w"), indent=1)
