// A/B policy variant ldsdma: plain one-wave launches load their columns through LDS (LDS-DMA)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.plain_lds_dma = 2;
    return p;
}();
