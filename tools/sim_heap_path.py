# The device loop's register-path heap push (pm_drl.hip path_push) restated in
# Python and checked against Go's container/heap (Push: up, Pop: swap + down) on
# random push/pop sequences with many equal keys: the array after every push
# must be identical.  python tools/sim_heap_path.py -> "ok"
import random
def go_push(h, x):
    h.append(x); j = len(h)-1
    while True:
        i = (j-1)//2
        if j == 0 or not (h[j][0] < h[i][0]): break
        h[i], h[j] = h[j], h[i]; j = i
def go_pop(h):
    n = len(h)-1; h[0], h[n] = h[n], h[0]
    i = 0
    while True:
        j1 = 2*i+1
        if j1 >= n: break
        j = j1
        if j1+1 < n and h[j1+1][0] < h[j1][0]: j = j1+1
        if not (h[j][0] < h[i][0]): break
        h[i], h[j] = h[j], h[i]; i = j
    return h.pop()
# the wave algorithm with the path in "lanes"
class Path:
    def __init__(self, hp, n):
        self.hp = hp; self.j = n+1
        self.pv = [None]*64
        for l in range(1, 32):
            a = self.j >> l
            self.pv[l] = hp[a-1] if a >= 1 else None
    def push(self, x):
        hp, j = self.hp, self.j; jn = j+1
        while len(hp) < j: hp.append(None)
        b = 0
        for l in range(1, 32):
            aj = j >> l
            if aj >= 1 and x[0] < self.pv[l][0]: b |= 1 << l
        c = 0
        while (b >> (c+1)) & 1: c += 1
        old = list(self.pv)
        writes = {}
        for l in range(1, c+1): writes[(j >> (l-1)) - 1] = old[l]
        writes[(j >> c) - 1] = x
        for k, v in writes.items(): hp[k] = v
        new = [None]*64
        for l in range(1, 32):
            aj = j >> l; an = jn >> l
            if an < 1: continue
            if an == aj:
                new[l] = old[l+1] if l < c else (x if l == c else old[l])
            elif an == (j >> (l-1)):
                l2 = l-1
                new[l] = old[l] if l2 < c else (x if l2 == c else old[l-1])
            else:
                new[l] = hp[an-1]
        self.pv = new; self.j = jn
random.seed(1)
for trial in range(3000):
    h = []; hp = []
    # mix of pushes and pops, with many ties
    P = None
    for step in range(random.randint(1, 400)):
        if h and random.random() < 0.3:
            a = go_pop(h); 
            # device pop on hp (same algorithm as go) then the path is reloaded
            b = go_pop(hp)
            assert a == b
            P = None
        else:
            x = (float(random.randint(0, 20)), step)
            go_push(h, x)
            if P is None: P = Path(hp, len(hp))
            P.push(x)
            assert hp[:len(h)] == h, (trial, step)
            del hp[len(h):]
print("ok")
