"""Integer model of the lazily reduced 28-bit G1 subgroup test (drand_amd/csrc/fp28.hpp), for tests/test_fp28_model.py.

Every value is the integer the device holds (14 normalised 28-bit limbs, Montgomery radix R' = 2^392). mont() is
fp_mul28.hpp mont_mul (exact integer (a b + m p) / R') and asserts the < 2p output bound the formulas rely on; lin()
is f28_lin and asserts the result stays in [0, 2^392); the formulas follow fp28.hpp line by line (j28_dbl, j28_madd,
j28_add, g1_in_subgroup28) and the 11-isogeny of the G1 hash (h2c.hpp iso11_jac). Test infrastructure only.
"""
p=0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
r=0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
RP=2**392; R=2**384
pinv=pow(p,-1,RP)
MAX=[0]
def mont(a,b):
    assert 0<=a<RP and 0<=b<RP
    t=a*b
    m=(-t*pinv)%RP
    o=(t+m*p)//RP
    assert o < 2*p, (a/p, b/p, o/p)
    return o
def lin(K,a,ca,b,cb):
    v=ca*a+cb*b+K*p
    assert 0<=v<RP, v/p
    MAX[0]=max(MAX[0], v/p)
    return v
def lin3(K,a,ca,b,cb,c,cc):
    v=ca*a+cb*b+cc*c+K*p
    assert 0<=v<RP, v/p
    MAX[0]=max(MAX[0], v/p)
    return v
add=lambda a,b: lin(0,a,1,b,1)
sub=lambda K,a,b: lin(K,a,1,b,-1)
scale=lambda a,c: lin(0,a,c,a,0)
ONE=RP%p
def zero(a): o=mont(a,1); return o==0 or o==p
def from_fp(x): # x is the normal field element
    xr=x*R%p
    return mont(xr, pow(2,400,p))
def sub_nc(K,a,b):
    # fp28.hpp f28_sub_nc<K>: a + K p - b limb by limb (redundant K p); every limb stays >= 0 when b's top limb is
    # below K p's
    assert (b>>(28*13)) < ((K*p)>>(28*13)), "f28_sub_nc: b's top limb reaches K p's"
    return lin(K,a,1,b,-1)
def dbl(P):
    # the subgroup test's inlined form (j28_dbl<true>): X + B and D + 32p - X3 feed their products carry-free
    # (f28_add_nc, f28_sub_nc<kp_above(26)>); its product bound covers the out-of-line form's D + 26p - X3
    X,Y,Z,fl=P
    a=mont(X,X); b=mont(Y,Y); c=mont(b,b); t=mont(add(X,b),add(X,b))
    d=lin3(8,t,2,a,-2,c,-2); e=scale(a,3); f=mont(e,e)
    x=lin(24,f,1,d,-2); m=mont(e,sub_nc(32,d,x)); y=lin(16,m,1,c,-8); z=scale(mont(Y,Z),2)
    return (x,y,z,fl)
def inf(): return (ONE,ONE,0,True)
def madd(P,qx,qy):
    X,Y,Z,fl=P
    if fl: return (qx,qy,ONE,False)
    z1z1=mont(Z,Z); u2=mont(qx,z1z1); s2=mont(mont(qy,Z),z1z1)
    h=sub(26,u2,X); rr=sub(18,s2,Y)
    if zero(h):
        return dbl(P) if zero(rr) else inf()
    hh=mont(h,h); i=scale(hh,4); j=mont(h,i); r2=scale(rr,2); v=mont(X,i)
    x=lin3(6,mont(r2,r2),1,j,-1,v,-2)
    m=mont(r2,sub(8,v,x)); y=lin(4,m,1,mont(Y,j),-2)
    zs=add(Z,h); z=lin3(4,mont(zs,zs),1,z1z1,-1,hh,-1)
    return (x,y,z,False)
def jadd(P,Q):
    X1,Y1,Z1,f1=P; X2,Y2,Z2,f2=Q
    if f1: return Q
    if f2: return P
    z1z1=mont(Z1,Z1); z2z2=mont(Z2,Z2); u1=mont(X1,z2z2); u2=mont(X2,z1z1)
    s1=mont(mont(Y1,Z2),z2z2); s2=mont(mont(Y2,Z1),z1z1)
    h=sub(2,u2,u1); rr=sub(2,s2,s1)
    if zero(h):
        return dbl(P) if zero(rr) else inf()
    h2=scale(h,2); i=mont(h2,h2); j=mont(h,i); r2=scale(rr,2); v=mont(u1,i)
    x=lin3(6,mont(r2,r2),1,j,-1,v,-2)
    m=mont(r2,sub(8,v,x)); y=lin(4,m,1,mont(s1,j),-2)
    zs=add(Z1,Z2); zz=lin3(4,mont(zs,zs),1,z1z1,-1,z2z2,-1); z=mont(zz,h)
    return (x,y,z,False)
U=0xd201000000010000
BETA=0x5f19672fdf76ce51ba69c6076a0f77eaddb3a93be6f89688de17d813620a00022e01fffffffefffe
def insub(px,py,beta):
    x=from_fp(px); y=from_fp(py)
    acc=(x,y,ONE,False)
    for b in range(62,-1,-1):
        acc=dbl(acc)
        if (U>>b)&1: acc=madd(acc,x,y)
    t=acc
    for b in range(62,-1,-1):
        acc=dbl(acc)
        if (U>>b)&1: acc=jadd(acc,t)
    X,Y,Z,fl=acc
    assert fl == zero(Z), "the infinity flag and Z = 0 disagree"
    if fl: return False
    bx=mont(from_fp(beta),x); z2=mont(Z,Z); z3=mont(z2,Z)
    if not zero(sub(26,mont(bx,z2),X)): return False
    return zero(add(mont(y,z3),Y))

def to_fp(a):  # f28_to_fp: one product by 2^384 mod p, then the final subtraction -> canonical x R mod p
    o=mont(a, R%p)
    return o-p if o>=p else o
def iso11(X32,Y32,Z32,xnum,xden,ynum,yden):
    """iso11_jac on a Jacobian point given in 12 x 32-bit Montgomery form (values x R mod p, canonical); coefficient
    lists low degree first as in RFC 9380 (normal field elements); returns (X', Y', Z') in the same form."""
    c=lambda v: v*RP%p
    f=lambda v: mont(v, pow(2,400,p))  # f28_from_fp on the stored value
    X=f(X32); Zp=f(Z32); D=mont(Zp,Zp)
    xn=c(xnum[-1]); xd=c(xden[-1]); yn=c(ynum[-1]); yd=c(yden[-1]); zp=D
    for j in range(1,len(ynum)):
        if j>1: zp=mont(zp,D)
        yn=add(mont(yn,X),mont(c(ynum[-1-j]),zp))
        yd=add(mont(yd,X),mont(c(yden[-1-j]),zp))
        if j<len(xnum): xn=add(mont(xn,X),mont(c(xnum[-1-j]),zp))
        if j<len(xden): xd=add(mont(xd,X),mont(c(xden[-1-j]),zp))
    a=mont(xd,D); z3=mont(D,Zp); ydz3=mont(yd,z3); rz=mont(a,ydz3)
    return (to_fp(mont(mont(xn,ydz3),rz)), to_fp(mont(mont(mont(f(Y32),yn),a),mont(rz,rz))), to_fp(rz))

# ---- the MSM's bucket additions (k_msm.hip MSM28): the same formulas without the exceptional-case tests, and the
# run-level zero test of Z that sends a poisoned run back through the exact formulas (fp28.hpp j28_madd_fast etc.)
def madd_fast(P,qx,qy):
    X,Y,Z,fl=P
    if fl: return (qx,qy,ONE,False)
    z1z1=mont(Z,Z); u2=mont(qx,z1z1); s2=mont(mont(qy,Z),z1z1)
    h=sub(26,u2,X); rr=sub(18,s2,Y)
    hh=mont(h,h); i=scale(hh,4); j=mont(h,i); r2=scale(rr,2); v=mont(X,i)
    x=lin3(6,mont(r2,r2),1,j,-1,v,-2)
    m=mont(r2,sub(8,v,x)); y=lin(4,m,1,mont(Y,j),-2)
    zs=add(Z,h); z=lin3(4,mont(zs,zs),1,z1z1,-1,hh,-1)
    return (x,y,z,False)
def jadd_fast(P,Q):
    X1,Y1,Z1,f1=P; X2,Y2,Z2,f2=Q
    if f1: return Q
    if f2: return P
    z1z1=mont(Z1,Z1); z2z2=mont(Z2,Z2); u1=mont(X1,z2z2); u2=mont(X2,z1z1)
    s1=mont(mont(Y1,Z2),z2z2); s2=mont(mont(Y2,Z1),z1z1)
    h=sub(2,u2,u1); rr=sub(2,s2,s1)
    h2=scale(h,2); i=mont(h2,h2); j=mont(h,i); r2=scale(rr,2); v=mont(u1,i)
    x=lin3(6,mont(r2,r2),1,j,-1,v,-2)
    m=mont(r2,sub(8,v,x)); y=lin(4,m,1,mont(s1,j),-2)
    zs=add(Z1,Z2); zz=lin3(4,mont(zs,zs),1,z1z1,-1,z2z2,-1); z=mont(zz,h)
    return (x,y,z,False)
def poisoned(P): return (not P[3]) and zero(P[2])
def neg2(y): return lin(2,y,-1,y,0)
def bucket_run(pts, affine):
    """k_msm_bucket28 on one run: pts = [(x28, y28) or (X, Y, Z) 28-bit, neg flag]; returns (sum, was_poisoned)."""
    acc=inf()
    for pt,neg in pts:
        if affine:
            x,y=pt; acc=madd_fast(acc,x,neg2(y) if neg else y)
        else:
            X,Y,Z=pt; acc=jadd_fast(acc,(X,neg2(Y) if neg else Y,Z,Z==0))
    if not poisoned(acc):
        return acc,False
    acc=inf()
    for pt,neg in pts:
        if affine:
            x,y=pt; acc=madd(acc,x,neg2(y) if neg else y)
        else:
            X,Y,Z=pt; acc=jadd(acc,(X,neg2(Y) if neg else Y,Z,Z==0))
    return acc,True
def to_affine(P):
    """normal-field affine point of a model Jacobian point (None = infinity)"""
    X,Y,Z,fl=P
    if fl: return None
    f=lambda v: v*pow(RP,-1,p)%p
    z=f(Z); zi=pow(z,-1,p)
    return (f(X)*zi*zi%p, f(Y)*zi**3%p)
