import numpy as np
f=np.float32
a=[f(4.89352455891786e-03),f(6.37261928875436e-04),f(1.48572235717979e-05),f(5.12229709037114e-08),f(-8.60467152213735e-11),f(2.00018790482477e-13),f(-2.76076847742355e-16)]
b=[f(4.89352518554385e-03),f(2.26843463243900e-03),f(1.18534705686654e-04),f(1.19825839466702e-06)]
def rat(x):
    x=np.clip(x,f(-7.90531110763549805),f(7.90531110763549805)).astype(f)
    x2=(x*x).astype(f)
    p=a[6]
    for c in a[5::-1]:
        p=(p*x2+c).astype(f)
    p=(p*x).astype(f)
    q=b[3]
    for c in b[2::-1]:
        q=(q*x2+c).astype(f)
    return (p/q).astype(f), p, q
x=np.concatenate([np.linspace(-10,10,2000001,dtype=np.float64), np.geomspace(1e-8,10,200001)]).astype(f)
r,p,q=rat(x)
ref=np.tanh(x.astype(np.float64))
rel=np.abs(r-ref)/np.maximum(np.abs(ref),1e-30)
print("max rel", rel.max(), "at", x[rel.argmax()], "max abs", np.abs(r-ref).max())
# with rcp approximated by 1-ulp error
