"""Rank-deficiency certificates for AMM updates, simulated on the oracle (round 4, DESIGN.md
§4.1): after a factorization that stops at rank k, w = [-S11^-1 S12 e_j; e_j] (j: the most
negative remaining diagonal) has w' Sigma w = S_jj < 0; counts how often the next update's Sigma
still satisfies w' Sigma w < -(Higham Thm 10.3 bound), i.e. is PROVEN rank deficient.

  python tools/cert_sim.py
"""
import sys, os, numpy as np
ROOT='/root/repo'; sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT,'tests'))
import _mamba_path, oracle_lib
mb=_mamba_path.load(); orc=oracle_lib.Oracle()
model=mb.rats(); model.setinputs(mb.model.RATS_DATA); model.setsamplers(mb.model.rats_scheme_gibbs_amm())
C=256; init=mb.model.rats_init_ls(16384, seed=1000)[:C]
st=orc.new_state(model, init)
d=30; T=d*(d+1)//2; tl=4+2*d+2*T; offs={"alpha":0,"beta":tl}
tri=np.array([i*(i+1)//2 for i in range(d)]); ii,kk=np.tril_indices(d)
u=2.0**-53; g31=31*u/(1-31*u); g36=36*u/(1-36*u)
orc.run(model, st, 128, seed=7, nthreads=8, draws=False)
W={b:[None]*C for b in offs}
stat={b:dict(n=0,deficient=0,cert=0,cert_wrong=0,had_w=0, q=[], ratio=[]) for b in offs}
for it in range(200):
    orc.run(model, st, 1, seed=7, nthreads=8, draws=False)
    for b,o in offs.items():
        t=st["tune"][:, o:o+tl]
        for c in range(C):
            m=t[c,1]; p=m/(m+1.0); Mv=t[c,4:4+d]; Mvv=t[c,4+d:4+d+T]; cc=(2.38*2.38/d)/p
            S=np.zeros((d,d)); vals=cc*(Mvv[tri[ii]+kk]-Mv[kk]*Mv[ii]); S[ii,kk]=vals; S[kk,ii]=vals
            r,_,piv=orc.pchol(S); piv=list(piv[:r])
            s=stat[b]; s["n"]+=1; defi = r<d; s["deficient"]+=defi
            w=W[b][c]
            if w is not None:
                s["had_w"]+=1
                q=w@S@w; aw=np.abs(w)
                marg=2*g31/(1-g31)*(aw@np.sqrt(np.abs(np.diag(S))))**2 + g36*(aw@np.abs(S)@aw)
                cert = q < -marg
                s["cert"]+=cert
                if cert and not defi: s["cert_wrong"]+=1
                if defi: s["q"].append(q); s["ratio"].append(-q/marg)
            if defi:
                if not (w is not None and (w@S@w) < -1e-9):
                    # new w from the partial factorization at the stop
                    rest=[e for e in range(d) if e not in piv]
                    if len(piv)>0:
                        S11=S[np.ix_(piv,piv)]; S12=S[np.ix_(piv,rest)]
                        X=np.linalg.solve(S11, S12)
                        Sch=S[np.ix_(rest,rest)]-S12.T@X
                    else:
                        X=np.zeros((0,len(rest))); Sch=S[np.ix_(rest,rest)]
                    j=int(np.argmin(np.diag(Sch)))
                    wn=np.zeros(d); wn[rest[j]]=1.0
                    if len(piv)>0: wn[piv]=-X[:,j]
                    W[b][c]=wn
            else:
                W[b][c]=None
for b,s in stat.items():
    q=np.array(s["ratio"])
    print(b, {k:v for k,v in s.items() if k not in ("q","ratio")}, "ratio pct", np.percentile(q,[0,1,50]) if len(q) else None)
