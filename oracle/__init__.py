"""CPU ORACLE for the CubeCobra DAE hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the *checker* (or the timed CPU
baseline) — never as the thing measured or shipped.  The product path
(``cubecobrarecommender_amd``) never imports it and fails loudly when its HIP
library is missing.

What is restated here (every function cites the reference file:line it follows):

* ``adjacency_ref``  — ``src/non_ml/utils.py:75-91`` (M) and ``src/ml/train.py:69-71`` (M~).
* ``noise_ref``      — ``src/ml/generator.py:6-103`` (F noise, reg-row sampling),
  twice: ``MTNoise`` replays the reference's own legacy-MT19937 draws bit-for-bit
  (pinned by golden vectors produced by importing the reference, see
  ``oracle/make_golden.py``), and ``philox_noise_batch`` is the same law driven by
  a counter-based Philox4x32-10 stream (the law the HIP kernel implements).
* ``model_ref``      — ``src/ml/model.py:20-125`` forward/backward with the TF-2.5
  Keras loss (``train.py:83-88``) and ResourceApplyAdam (``train.py:84``) formulas.
* ``infer_ref``      — ``src/scripts/ml_recommend.py:78-108`` /
  ``web/ml_recommend_web.py:39-64`` with a pinned fp32 summation order and a
  pinned tie rule, so top-N indices can be compared bit-exactly.

Parity status: the generator (MT19937 replay) and the adjacency matrix are pinned
against outputs of the reference code itself (``tests/golden``).  TensorFlow is not
installed anywhere in this pipeline, so the model/loss/optimizer arithmetic is a
restatement of TF 2.5.2's published formulas:
"parity unpinned" against TF itself.
"""
