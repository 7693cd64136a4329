# Test-infrastructure shim (NOT product code): just enough of PyG 2.3.1 for the reference's
# ET / NeighborEmbedding MessagePassing subclasses to run on CPU in this container.
