"""CPU oracle for the LPV-MPC hot path — TEST INFRASTRUCTURE ONLY (see ntm_oracle.py)."""
