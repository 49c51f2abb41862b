"""oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference MM-PDE forward path (Peiyannn/MM-PDE), used
as the parity checker by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and nowhere else.  Nothing in the product package imports it.

* refcpu.py      -- torch-CPU op-for-op restatement (gnn_2d.py, mesh/dmm_model.py,
                    interpolate.py, data_creator_2d.py, train_helper_2d.py).
* knn_oracle.c   -- C restatement of torch_cluster.knn_graph and sklearn kNN.

Parity status: torch-native ops pinned by torch itself; sklearn kNN-30 pinned
against sklearn 1.7.2 golden fixtures (tests/golden); torch_cluster knn_graph
and PyG/torch_scatter mean aggregation: "parity unpinned" (no reference
fixtures exist and running the reference was refused) --
pinned only by hand-derived KATs.
"""
