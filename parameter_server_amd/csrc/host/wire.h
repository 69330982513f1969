// Task frame (protobuf wire format, the reference's field numbers) for the
// fields of the filter path; see wire.cc.
#pragma once
#include <string>

#include "../psf_internal.h"
#include "message.h"

namespace psf {

std::string serialize_task(const Task& t);
// throws CheckError(kErrCheck) where protobuf's ParseFromArray would fail
void parse_task(const uint8_t* p, size_t n, Task* t);

}  // namespace psf
