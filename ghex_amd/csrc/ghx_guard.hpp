// ghx_guard.hpp — exception -> status conversion at the C ABI (no exception crosses it).
#pragma once

#include <hip/hip_runtime.h>

#include <new>
#include <string>

#include "ghx_plan.hpp"

namespace ghx
{
template<typename F>
int guarded(F&& f)
{
    try
    {
        set_error("");
        return f();
    }
    catch (const invalid& e)
    {
        set_error(e.what());
        return GHX_ERR_INVALID;
    }
    catch (const hip_error& e)
    {
        set_error(std::string(e.what()) + ": " + hipGetErrorString(hipGetLastError()));
        return GHX_ERR_HIP;
    }
    catch (const std::bad_alloc&)
    {
        set_error("out of host memory");
        return GHX_ERR_NOMEM;
    }
    catch (const std::exception& e)
    {
        set_error(e.what());
        return GHX_ERR_PATTERN;
    }
}

}  // namespace ghx
