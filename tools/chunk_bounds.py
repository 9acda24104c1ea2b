"""Per-layer bounds of one 625-pair LEF chunk: measured single-stream launch time (us, from
profiles/r02e_chunk_trace.txt, typed in below) against the algorithmic HBM bytes at 6 TB/s and the FLOPs at a
1.2 PFLOP/s practical MFMA ceiling; "gap" = time - max(bounds).  usage: python tools/chunk_bounds.py"""
P=625
L=[]  # name, t_us, M(out px per pair), K, N, in_px, in_ch, res(bool), x2 (in bytes extra)
s1=19*188; s2=10*94; s3=5*47; s4=3*24
def add(name,t,Mo,K,N,inpx,inch,res=False,extra_in=0):
    L.append((name,t,Mo,K,N,inpx,inch,res,extra_in))
add('stem',375.8,38*375,147,64,75*750,3)
add('s1.b0 fused',579.0,s1,None,None,s1,64)
add('s1.b1 fused',732.2,s1,None,None,s1,256)
add('s1.b2 fused',724.7,s1,None,None,s1,256)
add('s2.b0 red',341.2,s1,256,128,s1,256)
add('s2.b0 3x3s2',275.5,s2,1152,128,s1,128)
add('s2.b0 exp+sc',335,s2,384,512,s2,128,False,s1*256)
for b in (1,2,3):
    add(f's2.b{b} red',158,s2,512,128,s2,512)
    add(f's2.b{b} 3x3',240,s2,1152,128,s2,128)
    add(f's2.b{b} exp',267,s2,128,512,s2,128,True)
add('s3.b0 red',230,s2,512,256,s2,512)
add('s3.b0 3x3s2',240,s3,2304,256,s2,256)
add('s3.b0 sc',355,s3,512,1024,s2,512)
add('s3.b0 exp',145,s3,256,1024,s3,256,True)
for b in range(1,6):
    add(f's3.b{b} red',141,s3,1024,256,s3,1024)
    add(f's3.b{b} 3x3',211,s3,2304,256,s3,256)
    add(f's3.b{b} exp',160,s3,256,1024,s3,256,True)
add('s4.b0 red',230,s3,1024,512,s3,1024)
add('s4.b0 3x3s2',241,s4,4608,512,s3,512)
add('s4.b0 exp+sc',407,s4,1536,2048,s4,512,False,s3*1024)
for b in (1,2):
    add(f's4.b{b} red',138,s4,2048,512,s4,2048)
    add(f's4.b{b} 3x3',234,s4,4608,512,s4,512)
    add(f's4.b{b} exp',147,s4,512,2048,s4,512,True)
tot_t=tot_f=0; tot_lb=0
print(f"{'layer':14s} {'us':>6s} {'TF/s':>6s} {'GB':>6s} {'memus':>6s} {'mfmaus':>6s} {'gap':>5s}")
for name,t,Mo,K,N,inpx,inch,res,extra in L:
    if K is None:  # fused bottleneck
        cin=inch
        f=2*Mo*(cin*64+576*64+64*256+(64*256 if cin==64 else 0))*P
        by=(inpx*cin*2+Mo*256*2)*P
    else:
        f=2*Mo*K*N*P
        by=(inpx*inch*2+Mo*N*2+(Mo*N*2 if res else 0)+extra*2)*P
    mem=by/6.0e12*1e6; mf=f/1.2e15*1e6
    lb=max(mem,mf)
    tot_t+=t; tot_f+=f; tot_lb+=lb
    print(f"{name:14s} {t:6.0f} {f/t/1e6:6.0f} {by/1e9:6.2f} {mem:6.0f} {mf:6.0f} {t-lb:5.0f}")
print('total us',tot_t,'TF/s',tot_f/tot_t/1e6,'bound-sum',tot_lb)
