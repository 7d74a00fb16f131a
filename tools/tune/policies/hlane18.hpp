// A/B policy variant hlane18 (tools/ab_build.sh hlane18 -DELECT_EC_POLICY_HEADER=...)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hashed_scalar_base_min_cols = 99; p.hashed_lane_waves = 18;
    return p;
}();
