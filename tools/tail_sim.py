"""List-scheduling simulation of the search batch's tail ("The tail").  4096 persistent
searchers take queries from a counter; a query costs its expansions + 10 (init and descent), in
expansion units.  Compared: batch order, longest-first (LPT), and suspending a query after q
expansions (its continuation queued behind the fresh queries or ahead of them, re-queued while fresh
queries remain or always).  The per-query expansion counts come from the oracle's search on a
host-built SIFT-like graph (300k rows, ef 70, 10k queries), saved to /tmp/sift_cost.npy by:
  g = native.Graph.build(base, 0, 32, 100, 8, 100); view = oracle.IndexView(...);
  cost = [view.search(q, 10, 70, with_counters=True)[2][1] for q in queries]
"""
import numpy as np, heapq, collections, sys
c=np.load('/tmp/sift_cost.npy').astype(float)
W=4096; init=10.0
def ls(jobs):
    h=[0.0]*W
    for j in jobs:
        t=heapq.heappop(h); heapq.heappush(h,t+j)
    return max(h)
tot=(c+init).sum()/W
base=ls(c+init)
def policy(q, ovh, prefer_cont, only_while_fresh, maxsusp=99):
    fresh=collections.deque(c+init)
    cont=collections.deque()
    h=[(0.0,i) for i in range(W)]; heapq.heapify(h); end=0
    # running jobs: we need event sim where suspension pushes at time t+slice
    ev=[]  # (time, kind, worker, rem, nsusp)
    free=[(0.0,i) for i in range(W)]
    heapq.heapify(free)
    pending=[]  # continuations become available at time t (heap)
    t=0; done=0; n=len(c)
    events=[(0.0,i,None) for i in range(W)]  # worker free at time, with possibly a continuation to push
    heapq.heapify(events)
    while events:
        t,w,push=heapq.heappop(events)
        if push is not None: cont.append(push)
        job=None
        if prefer_cont and cont: job=cont.popleft()
        elif fresh: job=(fresh.popleft(),0)
        elif cont: job=cont.popleft()
        if job is None:
            end=max(end,t); continue
        rem,ns=job
        limit = q if ((not only_while_fresh) or fresh) and ns<maxsusp else 1e9
        if rem>limit:
            heapq.heappush(events,(t+limit+ovh,w,(rem-limit,ns+1)))
        else:
            heapq.heappush(events,(t+rem,w,None))
    # idle workers wait for cont: approximate (workers exit if nothing) -> need waiting; fix: re-run with waiting
    return end
def policy_wait(q, ovh, prefer_cont, only_while_fresh, maxsusp=99):
    fresh=collections.deque(c+init); cont=collections.deque()
    events=[(0.0,0,i,None) for i in range(W)]; heapq.heapify(events)
    idle=[]; end=0; seq=1
    while events:
        t,_,w,push=heapq.heappop(events)
        if push is not None:
            cont.append(push)
            # wake an idle worker
            while idle and cont:
                wi=idle.pop(); 
                heapq.heappush(events,(t,seq,wi,None)); seq+=1
        job=None
        if prefer_cont and cont: job=cont.popleft()
        elif fresh: job=(fresh.popleft(),0)
        elif cont: job=cont.popleft()
        if job is None:
            idle.append(w); end=max(end,t); continue
        rem,ns=job
        limit = q if ((not only_while_fresh) or fresh) and ns<maxsusp else 1e9
        if rem>limit:
            heapq.heappush(events,(t+limit+ovh,seq,w,(rem-limit,ns+1))); seq+=1
        else:
            heapq.heappush(events,(t+rem,seq,w,None)); seq+=1; end=max(end,t+rem)
    return end
print('batch', round(base/tot,3))
for q in (10,20,30,40,60,80):
  for ovh in (2,4):
    for pc in (False,True):
      for owf in (False,True):
        m=policy_wait(q,ovh,pc,owf)
        print(f'q{q} ovh{ovh} prefer_cont={pc} only_while_fresh={owf}: {m/tot:.3f} speedup {base/m:.3f}')
