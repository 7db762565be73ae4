"""Gilbert-equation physical model (README "Physical model", Readme.md:7-8).

The reference only declares it ("This classic model calculates oil flow using Gilbert's
equation"); BASELINE.json:7 keeps it as the CPU reference path. Gilbert (1954) critical
choke-flow correlation and its published re-fits, all of the form

    P_wh = A * R**B * q / S**C      =>      q = P_wh * S**C / (A * R**B)

q liquid rate [STB/d], P_wh wellhead (upstream) pressure [psig], S choke size [1/64 in],
R gas-liquid ratio (Mscf/STB for the Gilbert constant A = 435; scf/STB for the others).
Valid for critical flow (downstream/upstream pressure ratio <~ 0.55).

float64 numpy on the CPU, vectorised; it doubles as the ground truth of the synthetic
well-log generator (wellflow/data/synth.py) and as the non-learned baseline in the
val-MSE parity report.
"""
from __future__ import annotations

import dataclasses

import numpy as np

# name: (A, B, C, glr_unit) — glr_unit "mscf" means R in Mscf/STB, "scf" means scf/STB.
CORRELATIONS = {
    "gilbert": (435.0, 0.546, 1.89, "mscf"),
    "gilbert_scf": (10.0, 0.546, 1.89, "scf"),
    "ros": (17.40, 0.500, 2.00, "scf"),
    "baxendell": (9.56, 0.546, 1.93, "scf"),
    "achong": (3.82, 0.650, 1.88, "scf"),
}


@dataclasses.dataclass
class GilbertModel:
    correlation: str = "gilbert"
    max_pressure_ratio: float = 0.55  # critical-flow validity limit

    def constants(self):
        if self.correlation not in CORRELATIONS:
            raise ValueError(f"unknown correlation {self.correlation!r}; one of {sorted(CORRELATIONS)}")
        return CORRELATIONS[self.correlation]

    def flow_rate(self, whp, choke_64ths, glr_mscf):
        """q [STB/d] from wellhead pressure [psig], choke [1/64 in], GLR [Mscf/STB]."""
        A, B, C, unit = self.constants()
        p = np.asarray(whp, dtype=np.float64)
        s = np.asarray(choke_64ths, dtype=np.float64)
        r = np.asarray(glr_mscf, dtype=np.float64)
        if unit == "scf":
            r = r * 1000.0
        if np.any(r <= 0) or np.any(s <= 0):
            raise ValueError("choke size and GLR must be positive")
        return p * s**C / (A * r**B)

    def wellhead_pressure(self, q, choke_64ths, glr_mscf):
        """Inverse form: P_wh for a given rate."""
        A, B, C, unit = self.constants()
        r = np.asarray(glr_mscf, dtype=np.float64) * (1000.0 if unit == "scf" else 1.0)
        return A * r**B * np.asarray(q, np.float64) / np.asarray(choke_64ths, np.float64) ** C

    def is_critical(self, whp, downstream_pressure):
        return np.asarray(downstream_pressure) / np.asarray(whp) <= self.max_pressure_ratio

    # sklearn-like surface so the trainer can evaluate it like a learned model
    def predict(self, features: dict) -> np.ndarray:
        return self.flow_rate(features["whp"], features["choke"], features["glr"])

    def mse(self, features: dict, target) -> float:
        d = self.predict(features) - np.asarray(target, np.float64)
        return float(np.mean(d * d))
