// A/B policy variant ldsdma_read: read-heavy plain one-wave launches (decodes) load through LDS (LDS-DMA)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.plain_lds_dma = 1;
    return p;
}();
