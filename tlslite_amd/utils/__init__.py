"""tlslite-shaped cipher surface backed by the gfx950 kernels
(mirrors tlslite/utils/{cipherfactory,aes,rc4,tripledes}.py)."""
