"""Frame-time model of an early tail kernel for the slowest pixels of a cfg4 8-way shard (analysis only).

From the draw log of tools/chain_log.py (/tmp/chain_cfg4.npz): chains = shaded bounces per pixel;
the wavefront costs max(floor, n * unit) per iteration above tail_n live paths and tail_us per round
below (unit fitted to the measured 1-GPU frame); at iteration tf the K paths with the fewest samples
done move to a persistent tail kernel (fast_us per step) and the wavefront, slowed by infl, runs the
rest. Prints the modelled frame per (tf, K, infl)."""
import numpy as np, json
z=np.load('/tmp/chain_cfg4.npz'); d=z['draws'].astype(np.int32); b=((d-2)//7).astype(np.int64)
every=int(z['every']); W,H,spp=int(z['W']),int(z['H']),int(z['spp'])
chain=b.sum(1)
t1=1840.0; unit_ns=t1*1e6/(W*H*chain.mean())
floor_us=150.0; tail_n=17000; tail_us=42.0
def wave_time(ch):
    # ch: chains of the pixels in the wavefront (subsample); returns ms
    if len(ch)==0: return 0.0
    tmax=int(ch.max()); n=np.bincount(ch, minlength=tmax+1)
    alive=(len(ch)-np.cumsum(n))  # alive after t steps -> n(t) for t=0..
    alive=np.concatenate([[len(ch)],alive[:-1]])*every
    t=np.where(alive>tail_n, np.maximum(floor_us*1e-3, alive*unit_ns*1e-6), np.where(alive>0, tail_us*1e-3, 0))
    return float(t.sum()), np.cumsum(t)
base,cum=wave_time(chain)
print('base ms',round(base,1),'eff',round(t1/8/base,3))
# samples done after t steps: count of samples whose cumulative steps <= t
cs=np.cumsum(b,1)
for tf in (150,270,400,600):
    done=(cs<=tf).sum(1)
    rem=chain-tf
    for K in (256,768,1536,3072):
        k=max(1,K//every)
        alive=np.where(rem>0)[0]
        # predictor: fewest samples done (ties: more remaining? unknown) -> pick k
        order=alive[np.argsort(done[alive], kind='stable')]
        fast=order[:k]
        mask=np.ones(len(chain),bool); mask[fast]=False
        T_f=cum[tf-1] if tf>0 else 0
        wt,_=wave_time(chain[mask])
        for fast_us in (45.0,):
            tfast=T_f+rem[fast].max()*fast_us*1e-3
            for infl in (1.0,1.1):
                # wavefront after tf inflated by infl
                w2,c2=wave_time(chain[mask]); wt2=c2[tf-1]+(w2-c2[tf-1])*infl
                fr=max(wt2,tfast)
                print(json.dumps({"tf":tf,"K":K,"infl":infl,"T_f":round(T_f,1),"fast_end":round(tfast,1),"wave_end":round(wt2,1),"frame":round(fr,1),"eff":round(t1/8/fr,3),"oracle_gap":int(rem.max()-np.sort(rem)[-k-1])}))
