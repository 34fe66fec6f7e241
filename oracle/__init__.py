"""CPU restatement of the reference's Filter/Score pass — TEST INFRASTRUCTURE.

Two restatements live here:
  * ref_model.py   — object-level transcription of pkg/scheduler over
                     kubernetes_amd.api objects (pure Python, small cases only);
                     pinned by the golden vectors transcribed from the
                     reference's Go tests (tests/golden/).
  * ksg_oracle.c   — C restatement over the interned C-ABI inputs (faithful and
                     incremental modes), cross-checked against ref_model.py and
                     used as the GPU parity checker and bench.py's cpu_baseline.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package. The product (kubernetes_amd/) never imports it.
"""
