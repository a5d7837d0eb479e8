"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the SpotV2Net GAT hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package, and only as the checker / CPU baseline.  The product
(``spotv2net_amd``) never imports it and has no CPU path.

PARITY STATUS: **parity unpinned** against the reference implementation.
The arithmetic of the path lives in the third-party PyG 2.3.0
``torch_geometric.nn.GATConv`` (imported at reference utils/models.py:11,
version pinned only by prose at README.md:88 together with torch 2.2.2).  PyG
is not vendored under /root/reference, not installed in this image, and there
is no network to fetch it; the reference ships no tests, no golden vectors and
no stored notebook outputs.  The oracle therefore is:

* ``pyg_gatconv``  — an op-for-op restatement in PyTorch (CPU) of PyG 2.3.0
  GATConv (Linear/glorot init, remove_self_loops + add_self_loops
  fill_value='mean', edge_update, utils.softmax, propagate with aggr='add',
  concat/mean, bias) and of the reference's own GATModel
  (utils/models.py:61-152, which IS readable source);
* ``dense``        — an independent float64 numpy formulation of the same math
  (per graph, an n x n masked row softmax) used to cross-check the first;
* ``dataset``      — a restatement of CovarianceLaggedDataset.process
  (utils/dataset.py:182-289) in the reference's own numpy idiom.

What pins it: the two formulations agree, float64 gradcheck, known-answer
cases, and golden fixtures generated from it (tests/golden/make_golden.py).
"""
