"""ntm_mpc — MI355X-native batched LPV-MPC for NTM control (hot path of
IsaacSavona/MPC-NTM-Control's NTM_MPC_Sim.m receding-horizon loop).

Import requires nothing but the built HIP library at
``mpc-ntm-control_amd/lib/libntm_mpc.so``; see ``api.py``.
"""
from ._lib import (EXIT_INFEASIBLE, EXIT_MAXITER, EXIT_NONFINITE, EXIT_OPTIMAL, LIB_PATH, MODE_BOX,
                   MODE_FULL, MODE_FULL_DU, MODE_NONE, NtmLibraryError, load)
from .api import (Config, NtmMpc, NTM_MPC_Sim, Physics, Rho_to_PhiGammaLambda, device_tensor, is_scenario_major,
                  quadprog, rho1, rho2, rho3, scenarios_x0, ScenarioGen, scenario_sample)

__all__ = ["Config", "NtmMpc", "NTM_MPC_Sim", "Physics", "Rho_to_PhiGammaLambda", "quadprog", "rho1", "rho2",
           "rho3", "scenarios_x0", "ScenarioGen", "scenario_sample", "device_tensor", "is_scenario_major", "load", "LIB_PATH", "NtmLibraryError", "MODE_NONE", "MODE_BOX", "MODE_FULL", "MODE_FULL_DU",
           "EXIT_OPTIMAL", "EXIT_MAXITER", "EXIT_INFEASIBLE", "EXIT_NONFINITE"]
