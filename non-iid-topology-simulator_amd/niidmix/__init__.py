"""niidmix — MI355X-native neighbour parameter mixing for the non-IID topology simulator.

Hot path: one D-SGD round's Jacobi mixing Θ' = Wᵀ Θ over the [N, P] fp32 slab of all simulated
nodes (reference: tools/simulate/algorithm/d_sgd.py:96-116 over tools/setup/model/__init__.py:15-25).

Modules
  topology   topology.json reader (setup.topology.load mirror), CSR of Wᵀ, sparse MH builder
  factor     clique-factored form of W for D-Cliques (host, once per topology)
  ops        torch custom ops over libniidmix.so (HIP, gfx950) + Mixer (kernel selection)
  slab       NodeSlab: node models whose parameters are views into one [N, P] slab
  model      drop-in for setup.model.average
  d_sgd      drop-in algorithm plugin (optimizer / init / next_step / average / update_models)
  shard      multi-GPU: clique-aligned node shards + RCCL halo exchange

Importing niidmix.ops (or anything that launches kernels) loads libniidmix.so and fails loudly if
it is missing: there is no CPU fallback.
"""
__all__ = ["topology", "factor", "ops", "slab", "model", "d_sgd", "shard"]
