"""Trip-cost model of the lane loop (round 6): would deferring the interaction block
until more lanes need it -- each pending lane making its next step's depth-0 attempt speculatively -- pay?
Per-trip costs (fractions of a 21 k-cycle trip) from the GRM_TIMING attribution of profiles/r06_tabspec/
timing_attribution_r06a.log; a block costs its full length whenever any lane of the wave runs it (SIMT).
    python tools/defer_model.py
"""
import numpy as np
rng=np.random.default_rng(1)
# trip-cost model from the r06a timing attribution (fractions of a 21k-cycle trip):
C_PUSH=0.168+0.089   # attempt + restore/bookkeeping (runs if any lane attempts)
C_HEAD=0.128          # loop top + step head (stop test, photon_2, step size): runs if any lane begins a step
C_INT=0.142+0.200+0.105  # fluid + radiation + rest of interaction
C_TOP=0.081+0.035+0.030+0.012+0.010  # refill, tail, child, init, bias
F_FAIL=0.2; EXTRA=2.35   # P(first attempt of a step fails), extra attempts then (mean)
P_INT=0.95               # completed steps that need the interaction block
def sim(T, spec=True, trips=20000, L=64):
    # per lane: rem attempts of current step (1st attempt pending=1), depth0 flag, pending interaction
    rem=np.ones(L,int); first=np.ones(L,bool); pend=np.zeros(L,bool); done_wait=np.zeros(L,bool)
    cost=0.0; steps=0; ints=0
    for t in range(trips):
        # which lanes attempt this trip
        can = ~done_wait & ~(pend & ~first)   # pending lanes may only make depth-0 attempts
        if not spec: can &= ~pend
        att = can
        c = C_TOP
        if att.any(): c += C_PUSH
        if (att & first).any(): c += C_HEAD
        # outcome of attempts
        comp = np.zeros(L,bool)
        for i in np.where(att)[0]:
            if first[i]:
                if rng.random()<F_FAIL:
                    first[i]=False; rem[i]=int(rng.poisson(EXTRA-1))+2
                else: comp[i]=True
            else:
                rem[i]-=1
                if rem[i]<=0: comp[i]=True
        needs = comp & (rng.random(L)<P_INT)
        steps += comp.sum()
        # lanes completing while pending must wait for the round
        newly = needs & ~pend
        blocked = needs & pend
        done_wait |= blocked
        pend |= newly
        for i in np.where(comp)[0]: first[i]=True; rem[i]=1
        npend = pend.sum()
        if npend >= T or (not spec and npend>0 and False):
            c += C_INT; ints += 1
            pend[:] = False
            # lanes that were blocked: their completed step becomes pending now
            pend |= done_wait; done_wait[:] = False
        cost += c
    return steps/cost, ints/trips
base = sim(0.5, spec=True)  # T<1: interaction every trip (current design)
print('current (every trip)', round(base[0],2), 'steps per trip-cost')
for T in (32,40,48,56,60):
    r,f=sim(T)
    print(f'T={T}: steps/cost {r:.2f} ({r/base[0]-1:+.1%}), interaction rounds per trip {f:.2f}')
