import sys, math, numpy as np
sys.path.insert(0,'.')
import __graft_entry__ as ge
csm=ge._load_package()
w = csm.SyntheticWorld3D(num_nodes=2, num_submaps=1, world_x=20.0, world_y=20.0, world_z=5.0, num_boxes=8, max_range=14.0, seed=20250127 + 3)
c=int(w.submap_nodes[0]); cl=w.raw[c].astype(np.float64)
(tx,ty,tz),q=w.node_in_submap(c,0)
dyaw=math.radians(4.0)
q0=np.array([q[0]*math.cos(dyaw/2)-q[3]*math.sin(dyaw/2),0,0,q[3]*math.cos(dyaw/2)+q[0]*math.sin(dyaw/2)])
t0=np.array([tx+0.12,ty-0.08,tz+0.05])
def qmat(q):
    w_,x,y,z=q/np.linalg.norm(q)
    return np.array([[1-2*(y*y+z*z),2*(x*y-w_*z),2*(x*z+w_*y)],[2*(x*y+w_*z),1-2*(x*x+z*z),2*(y*z-w_*x)],[2*(x*z-w_*y),2*(y*z+w_*x),1-2*(x*x+y*y)]])
def aa(v):
    th=np.linalg.norm(v)
    if th==0: return np.eye(3)
    k=v/th; K=np.array([[0,-k[2],k[1]],[k[2],0,-k[0]],[-k[1],k[0],0]])
    return np.eye(3)+math.sin(th)*K+(1-math.cos(th))*K@K
R0=qmat(q0)
res=0.1; rmax=np.linalg.norm(cl,axis=1).max(); step=(1-1e-3)*math.acos(1-res*res/(2*rmax*rmax))
A=int(round(math.radians(15)/step)); print('A',A,'step',step)
cells=w.high_cells[0]; ijk=np.asarray(cells[0]).reshape(-1,3); lo=ijk.min(0)-1; hi=ijk.max(0)+1; dims=hi-lo+1; print('dims',dims)
rng=np.random.RandomState(0)
pts=cl[rng.choice(len(cl),400,replace=False)]
trans=np.array([[x,y,z] for z in range(-3,4) for y in range(-3,4) for x in range(-3,4)],float)*res
T=(R0@trans.T).T+t0
def lines(P, L):  # P: (..., 3) world points -> line ids
    c=np.clip(np.rint(P/res).astype(int)-lo,0,dims-1)
    lin=(c[...,2]*dims[1]+c[...,1])*dims[0]+c[...,0]
    return (lin*4)//L
for L in (64,128):
    # current: fixed rotation, wave = 64 consecutive translations
    cur=[]
    for trial in range(20):
        r=rng.randint(-A,A+1,3); R=R0@aa(r*step)
        rp=(R@pts.T).T
        for wv in range(0,343,64):
            tt=T[wv:wv+64]
            P=rp[:,None,:]+tt[None,:,:]
            cur.append(np.mean([len(np.unique(x)) for x in lines(P,L)]))
    new=[]
    for trial in range(20):
        r0=rng.randint(-A,A-3,3); tt=T[rng.randint(343)]
        Rs=[R0@aa((r0+np.array([a,b,cc]))*step) for a in range(4) for b in range(4) for cc in range(4)]
        P=np.stack([(R@pts.T).T+tt for R in Rs],1)
        new.append(np.mean([len(np.unique(x)) for x in lines(P,L)]))
    print(L,'B lines/instr: current (64 translations)',np.mean(cur),' rotations 4x4x4',np.mean(new))
