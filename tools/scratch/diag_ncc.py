import sys; sys.path[:0]=['oracle','sonido-sonar_amd']
import numpy as np, oracle as O, sonar
ctx=sonar.Context(0)
rng = np.random.default_rng(10000)
base = np.convolve(rng.standard_normal(5047), np.ones(5) / 5, "same")
a=base[37:5037]; b=base[:5000]
c,m=ctx.ncc(a,b,500); rc,rm=O.ncc(a,b,500)
d=np.abs(c-rc)/np.maximum(np.abs(rc),1e-300)
print('max rel', d.max(), 'n mismatch', np.sum(c!=rc), 'of', len(c), m['peak_lag'], rm['peak_lag'])
