// risc0/circuit/recursion/src/prove/hal/hip.rs — the recursion circuit's HAL over the HIP
// backend, beside the reference's cuda.rs in that directory (circuit/recursion/src/prove/hal/
// cuda.rs:40-190): witness generation, accumulation and eval_check on the device through the
// r0hip_* C ABI (include/r0hip.h), and the prover constructor the crate's `recursion_prover`
// selects. Not compiled here: the image has no Rust toolchain.
use std::rc::Rc;

use anyhow::Result;
use risc0_circuit_recursion_sys::RawPreflightTrace;
use risc0_core::field::baby_bear::{BabyBearElem, BabyBearExtElem};
use risc0_sys::ffi_wrap;
use risc0_zkp::hal::{hip::{BufferImpl, HipHash}, AccumPreflight, CircuitHal};
use risc0_zkp::zkp::StepMode;
use risc0_sys::hip::{r0hip_eval_check, r0hip_recursion_accum, r0hip_recursion_witgen};
use risc0_zkp::hal::hip::{HipHal, HipHashPoseidon2, HipHashPoseidon254, HipHashSha256};
use super::{CircuitAccumulator, CircuitWitnessGenerator, RecursionProver, RecursionProverImpl};
use crate::{REGISTER_GROUP_ACCUM, REGISTER_GROUP_CTRL, REGISTER_GROUP_DATA, GLOBAL_MIX, GLOBAL_OUT};

pub struct HipRecursionCircuitHal<HS: HipHash> { _hal: Rc<HipHal<HS>> }

impl<HS: HipHash> CircuitWitnessGenerator<HipHal<HS>> for HipRecursionCircuitHal<HS> {
    fn generate_witness(&self, _mode: StepMode, total_cycles: u32, preflight: &RawPreflightTrace,
                        ctrl: &BufferImpl<BabyBearElem>, data: &BufferImpl<BabyBearElem>,
                        global: &BufferImpl<BabyBearElem>) -> Result<()> {
        // on the device (r0hip_recursion_witgen: step_exec, the WOM sort and scan,
        // injectWomBacks and step_verify_mem of recursion-sys ffi.cpp:57-205, generated from
        // the reference's step code); the RawPreflightTrace arrays are host memory. The
        // result is the same for every StepMode, as the reference's modes agree.
        ffi_wrap(|| unsafe {
            r0hip_recursion_witgen(ctrl.dev(), data.dev(), global.dev(), total_cycles as usize,
                preflight.wom as *const u32, preflight.num_woms as usize,
                preflight.cycles as *const u32, preflight.num_cycles as usize,
                preflight.iops as *const u32, preflight.num_iops as usize)
        })
    }
}

impl<HS: HipHash> CircuitAccumulator<HipHal<HS>> for HipRecursionCircuitHal<HS> {
    // on the device: compute, prefix product and verify of recursion-sys ffi.cpp:160-217
    // (r0hip_recursion_accum, generated from the reference step code)
    fn accumulate(&self, work_cycles: u32, total_cycles: u32, ctrl: &BufferImpl<BabyBearElem>,
                  global: &BufferImpl<BabyBearElem>, data: &BufferImpl<BabyBearElem>,
                  mix: &BufferImpl<BabyBearElem>, accum: &BufferImpl<BabyBearElem>) -> Result<()> {
        ffi_wrap(|| unsafe {
            r0hip_recursion_accum(ctrl.dev(), global.dev(), data.dev(), mix.dev(), accum.dev(),
                                  work_cycles as usize, total_cycles as usize)
        })
    }
}

impl<HS: HipHash> CircuitHal<HipHal<HS>> for HipRecursionCircuitHal<HS> {
    fn eval_check(&self, check: &BufferImpl<BabyBearElem>, groups: &[&BufferImpl<BabyBearElem>],
                  globals: &[&BufferImpl<BabyBearElem>], poly_mix: BabyBearExtElem, po2: usize, _steps: usize) {
        let g = [groups[REGISTER_GROUP_ACCUM].dev() as *const u32, groups[REGISTER_GROUP_CTRL].dev() as *const u32,
                 groups[REGISTER_GROUP_DATA].dev() as *const u32];
        let pm = poly_mix.to_u32_words();
        ffi_wrap(|| unsafe { r0hip_eval_check(c"recursion".as_ptr(), check.dev(), g.as_ptr(),
            globals[GLOBAL_MIX].dev(), globals[GLOBAL_OUT].dev(), pm.as_ptr(), po2 as u32) }).unwrap();
    }
    // CircuitHal's preflight-driven accumulate: the recursion prover never calls it (it runs
    // CircuitAccumulator::accumulate above); the reference's CUDA HAL leaves it unimplemented
    // too (circuit/recursion/src/prove/hal/cuda.rs:174-185)
    fn accumulate(&self, _preflight: &AccumPreflight, _ctrl: &BufferImpl<BabyBearElem>, _io: &BufferImpl<BabyBearElem>,
                  _data: &BufferImpl<BabyBearElem>, _mix: &BufferImpl<BabyBearElem>, _accum: &BufferImpl<BabyBearElem>,
                  _steps: usize) {
        unimplemented!("the recursion prover accumulates through CircuitAccumulator")
    }
}

pub(crate) fn recursion_prover(hashfn: &str) -> Result<Box<dyn RecursionProver>> {
    macro_rules! with { ($hs:ty) => {{
        let hal = Rc::new(HipHal::<$hs>::new());
        let circuit_hal = Rc::new(HipRecursionCircuitHal { _hal: hal.clone() });
        Ok(Box::new(RecursionProverImpl::new(hal, circuit_hal)) as Box<dyn RecursionProver>)
    }}}
    match hashfn {
        "poseidon2" => with!(HipHashPoseidon2),
        "poseidon_254" => with!(HipHashPoseidon254),
        "sha-256" => with!(HipHashSha256),
        _ => anyhow::bail!("Unsupported hashfn: {hashfn}"),
    }
}
