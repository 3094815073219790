"""ORACLE - TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference (mshuaic/distributed-learning-contributivity) coalition-evaluation
path, used as the CHECKER by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
product package (distributed-learning-contributivity_amd/mplc) never imports anything from here.

Pinning (see DESIGN.md "Oracle"):
  shapley  - oracle_shapley_reference_order is bit-checked against the reference's own outputs
             (tests/golden/shapley_value.json, made by running mplc/contributivity.py:1210-1253).
  fedavg   - np.average restatement of mplc/mpl_utils.py:96-100, checked against the reference's
             FedAvg runs (tests/golden/fedavg_lr.json) through the LR path.
  cnn      - torch-CPU fp32 restatement of the Keras 2.3.1 MNIST CNN FedAvg semantics
             (mplc/dataset.py:457-479, mplc/multi_partner_learning.py:285-334).  The Keras/TF arithmetic
             cannot run in this image (no TF/Keras, no network): parity unpinned at the Keras boundary;
             anchored on the reference tests' accuracy thresholds (tests/end_to_end_tests.py:41-42,66-73).
"""
