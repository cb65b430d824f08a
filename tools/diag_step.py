"""Diagnostic: find teacher-forced steps where GPU and C oracle disagree; dump inputs."""
import sys, numpy as np, torch
import os
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'mpc-ntm-control_amd')]
from ntm_mpc import NtmMpc, Config
from oracle import ntm_oracle as O, cbind
ctl=NtmMpc()
dumps=[]
for (N,mode,B,ks) in [(20,2,48,12),(3,2,48,12),(50,1,48,4),(20,2,512,20)]:
    cfg=Config(N=N,mode=mode); ocfg=O.Config(N=N,mode=mode)
    x=O.scenario_x0(np.arange(B)).T.copy(); rho,Uo=cbind.initial_state(x,ocfg)
    bad=0; worst=0
    for k in range(ks):
        ref=cbind.step(x,rho,Uo,ocfg)
        out=ctl.step(torch.tensor(x,device='cuda'),torch.tensor(rho,device='cuda'),torch.tensor(Uo,device='cuda'),cfg)
        torch.cuda.synchronize()
        U=out['U'].cpu().numpy(); it=out['inner_iters'].cpu().numpy()
        e=np.max(np.abs(U-ref['U']),axis=0)/2e6
        worst=max(worst,e.max())
        for s in np.where((e>1e-10)|(it!=ref['inner_iters']))[0]:
            bad+=1
            if bad<=6: dumps.append(dict(N=N,mode=mode,k=k,s=int(s),x=x[:,s].copy(),rho=rho[:,s].copy(),Uo=Uo[:,s].copy(),Ugpu=U[:,s].copy(),Uref=ref['U'][:,s].copy(),itg=int(it[s]),itr=int(ref['inner_iters'][s])))
        x,rho,Uo=ref['x_next'],ref['rho'],ref['U_old']
    print(N,mode,B,"bad steps",bad,"worst",worst,flush=True)
np.save('gpurun_out/diag_dumps.npy',dumps,allow_pickle=True)
