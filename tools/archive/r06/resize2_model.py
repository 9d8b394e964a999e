"""Round 6: host-side model of k_pyr_resize2's index arithmetic (extractor_kernels.hip):
for each level pair, every level-l pixel is owned by exactly one tile, every
level-(l+1) tap lies inside the region the tile computes, and the LDS windows
fit (44 x 44 dwords for the level-l region, 56 x 56 for the level l-1 window).
Run: python3 tools/archive/r06/resize2_model.py -> [] per size = no pair rejected."""
import math, numpy as np
def tables(sw, dw):
    s = 1.0/(dw/sw)
    xo=[]
    for dx in range(dw):
        fx = np.float32((dx+0.5)*s-0.5); sx=int(math.floor(fx))
        if sx<0: sx=0
        if sx >= sw-1: sx = sw-1
        xo.append(sx)
    return xo
def levels(W,H,L=8,f=1.2):
    sc=[1.0]
    for i in range(1,L): sc.append(float(np.float32(sc[-1]*f)))
    out=[]
    for l in range(L):
        if l==0: out.append((W,H))
        else:
            inv=np.float32(1.0)/np.float32(sc[l])
            out.append((int(np.rint(np.float32(W)*inv)), int(np.rint(np.float32(H)*inv))))
    return out
def check(W,H,L=8,f=1.2):
    lv=levels(W,H,L,f)
    bad=[]
    for l in range(1,L-1):
        (w0,h0),(w1,h1),(w2,h2)=lv[l-1],lv[l],lv[l+1]
        xo1,yo1=tables(w0,w1),tables(h0,h1)
        xo2,yo2=tables(w1,w2),tables(h1,h2)
        covx=np.zeros(w1+4,int); covy=np.zeros(h1,int)
        ok=True
        for x0 in range(0,w2,128):
            xl=min(x0+127,w2-1); xt=min(x0+124,w2-1)
            X0=0 if x0==0 else xo2[x0]&~3
            ownX = w1 if x0+128>=w2 else xo2[x0+128]&~3
            X1e=max(min(xo2[xl]+1,w1-1)+1, ownX)
            nG1=(X1e-X0+3)>>2
            for g in range(nG1):
                if X0+4*g < ownX: covx[X0+4*g:X0+4*g+4]+=1
            # taps of T2 within R1
            for dx in range(x0, xl+1):
                assert X0 <= xo2[dx] and min(xo2[dx]+1,w1-1) < X0+4*nG1
            if nG1>44 or ((xo2[xt]-X0)>>2)+2>=44: ok=False
            c0a=xo1[X0]; c0b=min(xo1[min(X0+4*nG1-1,w1-1)]+1,w0-1)
            nW0=((c0b-(c0a&~3))>>2)+1
            if 4*((nW0+3)>>2)>56: ok=False
        for y0 in range(0,h2,32):
            yl=min(y0+31,h2-1)
            Y0=0 if y0==0 else min(max(yo2[y0],0),h1-1)
            ownY=h1 if y0+32>=h2 else min(max(yo2[y0+32],0),h1-1)
            Y1e=max(min(max(yo2[yl]+1,0),h1-1)+1,ownY)
            covy[Y0:ownY]+=1
            if Y1e-Y0>44: ok=False
            r0a=min(max(yo1[Y0],0),h0-1); r0b=min(max(yo1[Y1e-1]+1,0),h0-1)
            if r0b-r0a+1>56: ok=False
        assert (covx[:w1]==1).all(), (W,H,l,np.nonzero(covx[:w1]!=1)[0][:10])
        assert (covy==1).all(), (W,H,l)
        if not ok: bad.append(l)
    return bad
for W,H in [(1241,376),(640,480),(1920,1080),(752,480),(1226,370),(100,80),(4095,2000),(333,77)]:
    print(W,H,check(W,H))
print(check(1241,376,8,1.25), check(640,480,12,1.1))
