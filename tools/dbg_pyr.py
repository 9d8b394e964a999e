import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
import __graft_entry__ as g
orb=g.load_package(); import oracle
img=orb.synth_image(1,0,640,480)
ext=orb.ORBextractor(1000,1.2,8,20,7)
ext(img)
pyr=ext.mvImagePyramid; ref=oracle.pyramid(img)
for l,(a,b) in enumerate(zip(pyr,ref)):
    d=(a!=b)
    print(l,a.shape,d.sum(), np.argwhere(d)[:5].tolist() if d.any() else "")
    if d.any():
        y,x=np.argwhere(d)[0]; print("   gpu",a[y,x-2:x+6],"ref",b[y,x-2:x+6])
