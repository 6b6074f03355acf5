"""hsds_amd -- MI355X-native engine for the HSDS data-node chunk codec and hyperslab
gather/scatter hot path.

Modules:
  codec      storUtil-compatible _uncompress / _shuffle / _unshuffle (GPU)
  engine     batched device-resident decode and strided region copies
  selection  chunkUtil / dsetUtil selection math + GPU chunkReadSelection / chunkWriteSelection
  partition  chunk-id -> data node / GPU partitioning (idUtil)
"""
__version__ = "0.1.0"
