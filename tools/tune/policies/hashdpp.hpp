// A/B policy variant hashdpp: the parity hash weights lanes inside the DPP tree (wave_poly31)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hash_dpp_weights = true;
    return p;
}();
