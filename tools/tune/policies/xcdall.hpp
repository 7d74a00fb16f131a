// A/B policy variant xcdall: XCD-major block order (p.xcd_order = 2;)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.xcd_order = 2;
    return p;
}();
