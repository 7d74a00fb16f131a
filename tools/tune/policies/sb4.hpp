// A/B policy variant sb4: scalar stripe bases from 4 columns (RS(6,4) plain encode and decode)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.scalar_base_min_cols = 4;
    return p;
}();
