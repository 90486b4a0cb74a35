"""Structural fill of the 4x4 block sweep on the walker's H: column quads a round must
update, for the index pivot order and for the reverse-topological one."""
import os
import numpy as np, json
m=json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'allsteps_isaaclab_amd', 'model', 'walker3d.json')))
par=[l['parent'] for l in m['links']]
nl=len(par); NV=6+nl-1
# dof index: root 0..5, link i>=1 -> dof 5+i
def anc(i):
    s=set()
    while i>0: s.add(i); i=par[i]
    return s
dofl=lambda d: 0 if d<6 else d-5
Hs=np.zeros((28,28),bool)
for a in range(NV):
  for b in range(NV):
    la,lb=dofl(a),dofl(b)
    if la==0 or lb==0 or la in anc(lb) or lb in anc(la): Hs[a,b]=True
Hs[27,27]=True
def sim(order, blocks):
    S=Hs.copy(); tot=0; swept=set()
    pos=0
    for B in blocks:
        P=order[pos:pos+B]; pos+=B
        # columns with any nonzero in pivot rows (excluding pivot cols)
        cols=[j for j in range(28) if j not in P and S[P,:][:,j].any()]
        rows=[i for i in range(28) if i not in P and S[i,P].any()]
        tot+=len(cols)*B
        for i in rows:
            for j in cols: S[i,j]=True
        for i in range(28):
            for j in P: 
                if S[i,P].any() : pass
        print(B, 'cols',len(cols),'rows',len(rows))
    return tot
print('natural', sim(list(range(28)), [4]*7))
# leaf-first: arms R (links 14-17 -> dofs 19..22), arm L (23..26), leg R tail (hip_z,hip_y,knee,ankle: links 5-8 -> dofs 10..13), leg L tail (links 10-13 -> 15..18), then hip_x R (9), hip_x L (14), abd_x (8), abd_y(7), abd_z(6), root 0..5, pad 27
order=[19,20,21,22,23,24,25,26,10,11,12,13,15,16,17,18,9,14,8,7,6,0,1,2,3,4,5,27]
print('leaf', sim(order,[4]*7))
def simq(order, name):
    S=Hs.copy(); totq=0; tot=0
    for r in range(7):
        P=order[4*r:4*r+4]
        cols=[j for j in range(28) if j not in P and S[P,:][:,j].any()]
        quads=sorted(set(j//4 for j in cols))
        rows=[i for i in range(28) if i not in P and S[i,P].any()]
        for i in rows+P:
            for j in cols+P: S[i,j]=True
        totq+=len(quads); tot+=len(cols)
        print(r, P, 'cols', len(cols), 'quads', quads)
    print(name, 'cols', tot, 'quads', totq, 'of', 7*7)
simq(list(range(27,-1,-1)), 'reverse')
simq(list(range(28)), 'natural')
