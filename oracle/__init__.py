"""CPU oracle for the DistributedAUC hot path.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker; never by the product package
``distributedauc_amd``. See reference_cpu.py (Python/torch-CPU restatement) and
auc_oracle.c (plain-C restatement of the integer AUC counts and the fp32 update).
"""
