import sys, time, numpy as np, torch
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/mpc-ntm-control_amd')
from ntm_mpc import NtmMpc, Config, scenarios_x0
from oracle import ntm_oracle as O, cbind
ctl=NtmMpc()
for mode in (0,1,2):
    N=10 if mode==0 else 20
    cfg=Config(N=N, mode=mode); ocfg=O.Config(N=N, mode=mode)
    B=64
    x0=scenarios_x0(0,B) if mode else np.tile(O.REFERENCE_X0[:,None],(1,B))
    rho,Uo=cbind.initial_state(x0,ocfg)
    xk=x0.copy(); worst=0; flagmis=0
    for k in range(20):
        ref=cbind.step(xk,rho,Uo,ocfg)
        tx=torch.tensor(xk,device='cuda'); tr=torch.tensor(rho,device='cuda'); tu=torch.tensor(Uo,device='cuda')
        out=ctl.step(tx,tr,tu,cfg); torch.cuda.synchronize()
        e=np.max(np.abs(out['U'].cpu().numpy()-ref['U']))/2e6
        worst=max(worst,e); flagmis+=int((out['exitflag'].cpu().numpy()!=ref['exitflag']).sum())
        xk,rho,Uo=ref['x_next'],ref['rho'],ref['U_old']
    print("mode",mode,"teacher-forced worst U err",worst,"flag mismatches",flagmis, flush=True)
# timing
cfg=Config(N=20,mode=2); B=100000
x0=torch.tensor(scenarios_x0(0,B),device='cuda')
rho,Uo=ctl.initial_state(x0,cfg)
out=ctl.step(x0,rho,Uo,cfg); torch.cuda.synchronize()
t=time.time()
for k in range(3):
    out=ctl.step(out['x_next'].clone(),rho,Uo,cfg)
torch.cuda.synchronize(); dt=(time.time()-t)/3
print("B=1e5 step time %.3f s -> %.3e steps/s"%(dt,B/dt))
print("flags",torch.unique(out['exitflag'],return_counts=True))
