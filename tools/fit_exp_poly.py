import mpmath as mp
mp.mp.dps = 60
h = mp.log(2)/256
n = 4
# minimax for relative error of e^r with c0 = 1 fixed? Let Remez on f(r)=e^r, weight 1/e^r, full degree n.
def remez(n, a, b, iters=30):
    # initial Chebyshev alternation points
    m = n + 2
    xs = [ (a+b)/2 + (b-a)/2*mp.cos(mp.pi*i/(m-1)) for i in range(m)]
    xs.sort()
    for it in range(iters):
        # solve sum c_k x^k + (-1)^i E e^x = e^x
        A = mp.matrix(m, m); rhs = mp.matrix(m, 1)
        for i, x in enumerate(xs):
            for k in range(n+1): A[i,k] = x**k
            A[i, n+1] = (-1)**i * mp.e**x
            rhs[i] = mp.e**x
        sol = mp.lu_solve(A, rhs)
        c = [sol[k] for k in range(n+1)]; E = sol[n+1]
        err = lambda x: (sum(c[k]*x**k for k in range(n+1)) - mp.e**x)/mp.e**x
        # find extrema on fine grid
        N = 4000
        grid = [a + (b-a)*i/N for i in range(N+1)]
        vals = [err(x) for x in grid]
        # locate alternating extrema
        ext = [0]
        for i in range(1, N):
            if (vals[i]-vals[i-1])*(vals[i+1]-vals[i]) <= 0: ext.append(i)
        ext.append(N)
        if len(ext) != m:
            break
        xs = [grid[i] for i in ext]
    return c, max(abs(v) for v in vals)
c, e = remez(n, -h, h)
print('max rel err', mp.nstr(e, 5))
for k, ck in enumerate(c): print(k, repr(float(ck)), mp.nstr(ck - 1/mp.factorial(k), 5))
