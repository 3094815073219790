"""mplc (MI355X-native) - drop-in coalition-evaluation engine for MPLC's contributivity hot path.

Same public surface as the reference package's contributivity path (mplc.contributivity.Contributivity,
mplc.scenario.Scenario, mplc.multi_partner_learning.*); coalition values v(S) are computed by batched
HIP kernels in lib/libmplc_hip.so.  Unlike the reference (mplc/__init__.py:8-9),
importing the package has no side effects (no GPU memory cap, no logger setup).
"""
__version__ = "0.1.0"
