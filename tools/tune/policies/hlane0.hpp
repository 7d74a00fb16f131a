// A/B policy variant hlane0 (tools/ab_build.sh hlane0 -DELECT_EC_POLICY_HEADER=...)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hashed_scalar_base_min_cols = 99;
    return p;
}();
