// diffusion_mms — transient diffusion MMS with backward Euler through the MFEM-shaped host API,
// operators resident on the GPU across time steps.
//
// Follows myapps/convection_diffusion/diffusion_mms.cpp:
//   mass and LHS forms (M and M + alpha dt K) assembled once              :289-305
//   per step: rhs = M u_old (:430), rhs += dt (f(t), v) (:433-437), ProjectBdrCoefficient (:440-441),
//   FormLinearSystem (:444), PetscLinearSolver (:447-456), RecoverFEMSolution (:459)
//   exact u = sin(t) cos(2(x-1/2)^2 + 2(y-1/2)^2), f = u_t - alpha Lap u  (:136-178)
// On the GPU both operators stay resident; FormLinearSystem per step is B = b - A x_e, B_ess = x_ess
// on the already-eliminated operator (no re-assembly, no RAP as hypre does at :444).
//
//   diffusion_mms [-mesh file.msh | -n elems] [-p order] [-a alpha] [-dt dt] [-T t_final] [-opts petsc.opts]
// Output: dofs, steps, final_l2, gmres_iterations, seconds_per_step.  Exit code 3 on error.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <string>

#include "cdfem_mfem.hpp"

using namespace cdfem::mfem;

namespace {

class ExactCoefficient : public Coefficient {
public:
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const double dx = x[0] - 0.5, dy = x[1] - 0.5;
        return std::sin(GetTime()) * std::cos(2.0 * dx * dx + 2.0 * dy * dy);
    }
};

class ForcingCoefficient : public Coefficient {
public:
    explicit ForcingCoefficient(double alpha) : alpha_(alpha) {}
    real_t Eval(ElementTransformation &T, const IntegrationPoint &ip) override
    {
        Vector x;
        T.Transform(ip, x);
        const double t = GetTime(), dx = x[0] - 0.5, dy = x[1] - 0.5;
        const double r2 = dx * dx + dy * dy, q = 2.0 * r2;
        const double ut = std::cos(t) * std::cos(q);
        const double lap = std::sin(t) * (-16.0 * r2 * std::cos(q) - 8.0 * std::sin(q));
        return ut - alpha_ * lap;
    }

private:
    double alpha_;
};

}  // namespace

int main(int argc, char **argv)
{
    try {
        std::string mesh_file, opts;
        int n = 16, order = 1;
        double alpha = 0.1, dt = 0.05, t_final = 2.0;  // Input/input_diffusion_mms.yaml
        for (int i = 1; i + 1 < argc; i += 2) {
            const std::string k = argv[i];
            const char *v = argv[i + 1];
            if (k == "-mesh") mesh_file = v;
            else if (k == "-n") n = std::atoi(v);
            else if (k == "-p") order = std::atoi(v);
            else if (k == "-a") alpha = std::atof(v);
            else if (k == "-dt") dt = std::atof(v);
            else if (k == "-T") t_final = std::atof(v);
            else if (k == "-opts") opts = v;
            else throw std::invalid_argument("unknown option " + k);
        }
        MFEMInitializePetsc(&argc, &argv, opts.empty() ? nullptr : opts.c_str(), nullptr);
        Mesh mesh = mesh_file.empty() ? Mesh::MakeCartesian2D(n, n, Element::QUADRILATERAL) : Mesh(mesh_file.c_str(), 1, 1);
        H1_FECollection fec(order, mesh.Dimension());
        ParFiniteElementSpace fespace(&mesh, &fec);
        Array<int> ess_bdr(mesh.bdr_attributes.Max());
        ess_bdr = 1;
        Array<int> ess_tdof_list;
        fespace.GetEssentialTrueDofs(ess_bdr, ess_tdof_list);

        ExactCoefficient exact_coeff;
        ForcingCoefficient forcing_coeff(alpha);
        ConstantCoefficient alpha_dt_coeff(alpha * dt);

        ParBilinearForm mass_form(&fespace);
        mass_form.AddDomainIntegrator(new MassIntegrator());
        mass_form.Assemble();
        mass_form.Finalize();
        ParBilinearForm lhs_form(&fespace);
        lhs_form.AddDomainIntegrator(new MassIntegrator());
        lhs_form.AddDomainIntegrator(new DiffusionIntegrator(alpha_dt_coeff));
        lhs_form.Assemble();
        lhs_form.Finalize();

        ParGridFunction u(&fespace);
        exact_coeff.SetTime(0.0);
        u.ProjectCoefficient(exact_coeff);

        const int nsteps = static_cast<int>(std::ceil(t_final / dt - 1.0e-12));
        Vector rhs_local(fespace.GetVSize());
        OperatorHandle Ah(Operator::Hypre_ParCSR);
        Vector X, B;
        long gmres_its = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int step = 1; step <= nsteps; step++) {
            const double t = step * dt;
            mass_form.Mult(u, rhs_local);
            forcing_coeff.SetTime(t);
            ParLinearForm f_form(&fespace);
            f_form.AddDomainIntegrator(new DomainLFIntegrator(forcing_coeff));
            f_form.Assemble();
            rhs_local.Add(dt, f_form);
            exact_coeff.SetTime(t);
            u.ProjectBdrCoefficient(exact_coeff, ess_bdr);
            lhs_form.FormLinearSystem(ess_tdof_list, u, rhs_local, Ah, X, B);
            HypreParMatrix *A_hyp = Ah.As<HypreParMatrix>();
            if (!A_hyp) throw std::runtime_error("Expected HypreParMatrix.");
            PetscParMatrix A_petsc(0, A_hyp, Operator::PETSC_MATAIJ);
            PetscLinearSolver solver(A_petsc);
            solver.SetPrintLevel(0);
            solver.Mult(B, X);
            if (!solver.GetConverged())
                throw std::runtime_error("PETSc solver did not converge at step " + std::to_string(step));
            gmres_its += solver.GetNumIterations();
            lhs_form.RecoverFEMSolution(X, rhs_local, u);
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double t_end = nsteps * dt;
        exact_coeff.SetTime(t_end);
        const int order_quad = std::max(2, 2 * order + 3);
        const IntegrationRule *irs[Geometry::NumGeom] = {};
        for (int g = 0; g < Geometry::NumGeom; ++g) irs[g] = &IntRules.Get(g, order_quad);
        const double final_l2 = u.ComputeL2Error(exact_coeff, irs);
        std::printf("dofs %d\nsteps %d\nfinal_l2 %.17g\ngmres_iterations %ld\nseconds_per_step %.6g\n",
                    fespace.GetTrueVSize(), nsteps, final_l2, gmres_its, secs / std::max(nsteps, 1));
        MFEMFinalizePetsc();
        return 0;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
}
